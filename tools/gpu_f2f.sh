#!/bin/bash
# Writer/CLI pass: golden CLI tests (thread and process writers), then the file-to-file runs.
#   gpurun --timeout 900 -- bash tools/gpu_f2f.sh TAG
set -e -o pipefail
TAG=${1:-f2f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "golden or cli" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u tools/file_bench.py --config C2 --n_mg 10000 > "$OUT/f2f_c2.json" 2> "$OUT/f2f_c2.err" || { tail -20 "$OUT/f2f_c2.err"; exit 1; }
cat "$OUT/f2f_c2.json"
timeout -k 10 400 python -u tools/file_bench.py --config C2 --tiny --n_mg 100000 > "$OUT/f2f_tiny100k.json" 2> "$OUT/f2f_tiny100k.err" || { tail -20 "$OUT/f2f_tiny100k.err"; exit 1; }
cat "$OUT/f2f_tiny100k.json"
