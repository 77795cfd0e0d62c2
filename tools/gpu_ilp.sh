#!/bin/bash
# run_ilp pass: its GPU tests (then optionally the ILP bench).
#   gpurun --timeout 600 -- bash tools/gpu_ilp.sh TAG [bench]
set -e -o pipefail
TAG=${1:-ilp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ilp.py -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -8 "$OUT/pytest_gpu.log"
if [ "${2:-}" = bench ]; then
  timeout -k 10 300 python -u tools/ilp_bench.py > "$OUT/ilp_bench.json" 2> "$OUT/ilp_bench.err" || { tail -20 "$OUT/ilp_bench.err"; exit 1; }
  cat "$OUT/ilp_bench.json"
fi
