#!/bin/bash
# r04y: ILP GPU tests with their printed statuses, gaps and solve times (final library).
set -e -o pipefail
mkdir -p gpurun_out/r04y
timeout -k 10 600 python -u -m pytest tests/test_ilp.py -m gpu -q --timeout 400 --timeout-method thread \
  -rA -s > gpurun_out/r04y/ilp.log 2>&1 || { tail -40 gpurun_out/r04y/ilp.log; exit 1; }
grep -E "C3|C5|full|ILP|inexact|passed|failed" gpurun_out/r04y/ilp.log | tail -16
