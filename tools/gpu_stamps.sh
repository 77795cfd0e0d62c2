#!/bin/bash
# Per-phase stamps (diagnostic build) for the given configs.
#   gpurun --timeout 300 -- bash tools/gpu_stamps.sh TAG "C2:10000 C4:4000"
set -e -o pipefail
TAG=${1:-stamps}; CFGS=${2:-"C2:10000 C4:4000"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for cn in $CFGS; do
  C=${cn%%:*}; N=${cn##*:}
  REPIC_GC_LIB=repic-copy_amd/repic_amd/librepic_gc_diag.so timeout -k 10 200 \
    python -u tools/phase_stamps.py $C $N > "$OUT/stamps_$C.txt" 2>&1 || { tail -20 "$OUT/stamps_$C.txt"; exit 1; }
  cat "$OUT/stamps_$C.txt"
done
