#!/bin/bash
# r04i: phase timing (stop builds) + variant A/B on C2 / C4, then per-phase VALU / lane PMC of
# the stop builds and the variants on C2.
set -e -o pipefail
mkdir -p gpurun_out/r04i
for C in "C2 10000 7" "C4 12500 5"; do
  set -- $C
  timeout -k 10 400 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04i/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04i/ab_$1.txt; exit 1; }
  cat gpurun_out/r04i/ab_$1.txt
done
timeout -k 10 600 bash tools/gpu_pmc_ablate.sh r04i/pmc_stop C2 10000 lane > gpurun_out/r04i/pmc_stop.log 2>&1
cat gpurun_out/r04i/pmc_stop/delta.txt
LIBS="abl/librepic_gc_z*.so" timeout -k 10 400 bash tools/gpu_pmc_ablate.sh r04i/pmc_var C2 10000 lane > gpurun_out/r04i/pmc_var.log 2>&1
grep -E "==|SQ_INSTS_VALU|THREAD_CYCLES|ACTIVE_INST" gpurun_out/r04i/pmc_var/summary.log
