#!/bin/bash
# r04o: SQ issue/stall counters (r03 library vs product) on C2, then the driver's bench line.
set -e -o pipefail
mkdir -p gpurun_out/r04o
LIBS="abl/librepic_gc_zprev.so" timeout -k 10 300 bash tools/gpu_pmc_ablate.sh r04o/pmc C2 10000 > gpurun_out/r04o/pmc.log 2>&1 || { tail -30 gpurun_out/r04o/pmc.log; exit 1; }
cat gpurun_out/r04o/pmc/summary.log
bash tools/gpu_bench_byconfig.sh r04o/bc
