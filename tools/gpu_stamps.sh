#!/bin/bash
# Per-phase s_memtime shares and the workgroup timeline of the fused kernel (diagnostic build
# librepic_gc_diag.so, built on the CPU side with `make -C repic-copy_amd/csrc diag`).
#   gpurun --timeout 300 -- bash tools/gpu_stamps.sh TAG [CONFIG:N_MG ...]
set -e -o pipefail
TAG=${1:-stamps}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
CFGS=${*:-C2:10000}
for cn in $CFGS; do
  C=${cn%%:*}; N=${cn##*:}
  timeout -k 10 120 python -u tools/phase_stamps.py "$C" "$N" > "$OUT/stamps_$C.txt" 2>&1 \
    || { tail -20 "$OUT/stamps_$C.txt"; exit 1; }
  cat "$OUT/stamps_$C.txt"
done
