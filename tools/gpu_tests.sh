#!/bin/bash
# GPU parity tests only (one process, per-test timeout), optionally a test selection.
#   gpurun --timeout 900 -- bash tools/gpu_tests.sh TAG [pytest args...]
set -e -o pipefail
TAG=${1:-tests}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --durations=15 "$@" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -25 "$OUT/pytest_gpu.log"
