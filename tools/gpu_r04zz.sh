#!/bin/bash
# Per-phase VALU / lane efficiency of the final library (stop builds under abl/) on C2 and C4.
set -e -o pipefail
mkdir -p gpurun_out/r04zz
timeout -k 10 500 bash tools/gpu_pmc_ablate.sh r04zz/c2 C2 10000 lane > gpurun_out/r04zz/c2.log 2>&1 || { tail -30 gpurun_out/r04zz/c2.log; exit 1; }
cat gpurun_out/r04zz/c2/delta.txt
timeout -k 10 500 bash tools/gpu_pmc_ablate.sh r04zz/c4 C4 12500 lane > gpurun_out/r04zz/c4.log 2>&1 || { tail -30 gpurun_out/r04zz/c4.log; exit 1; }
cat gpurun_out/r04zz/c4/delta.txt
