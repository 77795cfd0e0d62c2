#!/bin/bash
# score_detections pass: its GPU tests, then the throughput line.
#   gpurun --timeout 600 -- bash tools/gpu_score.sh TAG
set -e -o pipefail
TAG=${1:-score}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_score.py tests/test_host_native.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -8 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u tools/score_bench.py > "$OUT/score_bench.json" 2> "$OUT/score_bench.err" || { tail -20 "$OUT/score_bench.err"; exit 1; }
cat "$OUT/score_bench.json"
