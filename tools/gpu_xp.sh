#!/bin/bash
# Timing-only experiment pass: tools/ablate.py on each CONFIG (every library under
# abl/ plus the product build, interleaved in one process), then once more per
# RGC_DIAG_NT value (workgroup size forced for every library).  No parity tests.
#   gpurun --timeout 600 -- bash tools/gpu_xp.sh TAG "C2 C4" "256"
set -e -o pipefail
TAG=${1:-xp}; CFGS=${2:-C2}; NTS=${3:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for C in $CFGS; do
  N=10000; [ "$C" = "C4" ] && N=4000; [ "$C" = "C3" ] && N=2000; [ "$C" = "C5" ] && N=16
  timeout -k 10 240 python -u tools/ablate.py "$C" "$N" 7 > "$OUT/ab_$C.txt" 2>&1 \
    || { tail -20 "$OUT/ab_$C.txt"; exit 1; }
  cat "$OUT/ab_$C.txt"
  for NT in $NTS; do
    RGC_DIAG_NT=$NT timeout -k 10 240 python -u tools/ablate.py "$C" "$N" 7 > "$OUT/ab_${C}_nt$NT.txt" 2>&1 \
      || { tail -20 "$OUT/ab_${C}_nt$NT.txt"; exit 1; }
    echo "RGC_DIAG_NT=$NT"; cat "$OUT/ab_${C}_nt$NT.txt"
  done
done
