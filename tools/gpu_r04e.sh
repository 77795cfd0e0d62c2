#!/bin/bash
# r04e: A/B timing (HEAD build abl/librepic_gc_zprev.so vs the working tree's product build and
# its variants) on C2 / C4 / C5, then GPU tests of the product build (ILP search with the
# Lagrangian bound, lazy stats, goldens, large route).
set -e -o pipefail
bash tools/gpu_ab3.sh r04e
mkdir -p gpurun_out/r04e
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -k "ilp or submit or golden or large_route or c5 or bench_step or smoke" -rA \
  > gpurun_out/r04e/pytest.log 2>&1 || { tail -60 gpurun_out/r04e/pytest.log; exit 1; }
grep -E "C3|C5|passed|failed" gpurun_out/r04e/pytest.log | tail -20
