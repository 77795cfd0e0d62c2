#!/bin/bash
# r04f: A/B of the round-4 fused-kernel changes one by one (abl/ variants) on C2/C4/C5, then
# the ILP GPU tests with their printed statuses / gaps.
set -e -o pipefail
bash tools/gpu_ab3.sh r04f
timeout -k 10 600 python -u -m pytest tests/test_ilp.py -m gpu -q --timeout 400 --timeout-method thread \
  -rA -s > gpurun_out/r04f/ilp.log 2>&1 || { tail -60 gpurun_out/r04f/ilp.log; exit 1; }
grep -E "C3|C5|full|passed|failed" gpurun_out/r04f/ilp.log | tail -30
