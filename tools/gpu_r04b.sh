#!/bin/bash
# r04b: ILP/smoke tests + driver bench with by_config, then per-phase lane efficiency (PMC).
set -e -o pipefail
bash tools/gpu_bench_byconfig.sh r04b "ilp or smoke"
timeout -k 10 400 bash tools/gpu_pmc_ablate.sh r04b_lane C2 10000 lane > gpurun_out/r04b_lane.log 2>&1 \
  || { tail -30 gpurun_out/r04b_lane.log; exit 1; }
cat gpurun_out/r04b_lane/delta.txt
