#!/bin/bash
# r04c: parity of the candidate build (abl/librepic_gc_ztri.so: K = 3 triangle pass, detached
# kernel arguments, large-route per-picker grids), then A/B timing on C2, C4 and C5.
set -e -o pipefail
mkdir -p gpurun_out/r04c
REPIC_GC_LIB=$PWD/abl/librepic_gc_ztri.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "golden or oracle or dense or bench_step or full_c2 or large_route or c5 or mixed or device_resident or submit or ilp" \
  > gpurun_out/r04c/tri_pytest.log 2>&1 || { tail -40 gpurun_out/r04c/tri_pytest.log; exit 1; }
tail -2 gpurun_out/r04c/tri_pytest.log
for C in "C2 10000 7" "C4 12500 5" "C5 64 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04c/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04c/ab_$1.txt; exit 1; }
  cat gpurun_out/r04c/ab_$1.txt
done
