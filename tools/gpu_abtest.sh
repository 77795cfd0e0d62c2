#!/bin/bash
# A/B pass: selected parity tests on the product build, then interleaved timing of every
# library under abl/ + the product build on C2 and C4.
#   gpurun --timeout 600 -- bash tools/gpu_abtest.sh TAG "pytest -k expr"
set -e -o pipefail
TAG=${1:-abtest}; KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 200 python -u tools/ablate.py C2 10000 7 > "$OUT/ab_c2.txt" 2>&1
cat "$OUT/ab_c2.txt"
timeout -k 10 200 python -u tools/ablate.py C4 4000 7 > "$OUT/ab_c4.txt" 2>&1
cat "$OUT/ab_c4.txt"
