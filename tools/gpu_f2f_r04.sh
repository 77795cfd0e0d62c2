#!/bin/bash
# File-to-file rates per config (never the bench value): the CLI on BOX text,
# one GPU, C2 10k, C3 4k, C4 12.5k (the 100k / 8-GPU shard), C5 64.
#   gpurun --timeout 1200 -- bash tools/gpu_f2f_r04.sh TAG
set -e -o pipefail
TAG=${1:-f2f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in "C2 10000" "C3 4000" "C4 12500" "C5 64"; do
  set -- $C
  timeout -k 10 400 python -u tools/file_bench.py --config $1 --n_mg $2 > "$OUT/f2f_$1.json" 2> "$OUT/f2f_$1.err" \
    || { tail -20 "$OUT/f2f_$1.err"; exit 1; }
  cat "$OUT/f2f_$1.json"
done
