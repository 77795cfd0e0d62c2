#!/bin/bash
# r04b: ILP/smoke tests + driver bench with by_config (product), per-phase lane efficiency
# (PMC), parity of the candidate build (abl/librepic_gc_ztri.so: K = 3 triangle pass, large-route
# per-picker grids), A/B timing on C2 and C5.
set -e -o pipefail
bash tools/gpu_bench_byconfig.sh r04b "ilp or smoke"
timeout -k 10 400 bash tools/gpu_pmc_ablate.sh r04b_lane C2 10000 lane > gpurun_out/r04b_lane.log 2>&1 \
  || { tail -30 gpurun_out/r04b_lane.log; exit 1; }
cat gpurun_out/r04b_lane/delta.txt
REPIC_GC_LIB=$PWD/abl/librepic_gc_ztri.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "golden or oracle or dense or bench_step or full_c2 or large_route or c5 or mixed" \
  > gpurun_out/r04b_tri_pytest.log 2>&1 || { tail -40 gpurun_out/r04b_tri_pytest.log; exit 1; }
tail -2 gpurun_out/r04b_tri_pytest.log
mkdir -p gpurun_out/r04b_ab
timeout -k 10 300 python -u tools/ablate.py C2 10000 7 > gpurun_out/r04b_ab/c2.txt 2>&1 || { tail -20 gpurun_out/r04b_ab/c2.txt; exit 1; }
cat gpurun_out/r04b_ab/c2.txt
rm -f abl/librepic_gc_stop*.so
timeout -k 10 300 python -u tools/ablate.py C5 64 5 > gpurun_out/r04b_ab/c5.txt 2>&1 || { tail -20 gpurun_out/r04b_ab/c5.txt; exit 1; }
cat gpurun_out/r04b_ab/c5.txt
