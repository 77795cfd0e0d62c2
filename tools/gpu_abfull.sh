#!/bin/bash
# Full GPU parity suite on the product build, then interleaved A/B timing of every library
# under abl/ + the product build on C2, C4 and C3.  First failure ends the script.
#   gpurun --timeout 900 -- bash tools/gpu_abfull.sh TAG
set -e -o pipefail
TAG=${1:-abfull}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for cn in C2:10000 C4:4000 C3:1000; do
  C=${cn%%:*}; N=${cn##*:}
  timeout -k 10 200 python -u tools/ablate.py $C $N 7 > "$OUT/ab_$C.txt" 2>&1 || { tail -20 "$OUT/ab_$C.txt"; exit 1; }
  cat "$OUT/ab_$C.txt"
done
