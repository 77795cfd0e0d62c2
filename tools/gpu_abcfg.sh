#!/bin/bash
# A/B timing of every abl/*.so against the product build (tools/ablate.py: device ms per step,
# interleaved in one process per config, median of ROUNDS), then optionally the phase stamps
# of the diagnostic build.  Experiments only: no parity tests.
#   gpurun --timeout 600 -- bash tools/gpu_abcfg.sh TAG "C2:10000:7 C4:12500:5" [stamps CFG:N ...]
set -e -o pipefail
TAG=${1:-ab}
CFGS=${2:-C2:10000:7}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for cn in $CFGS; do
  IFS=: read -r C N R <<< "$cn"
  timeout -k 10 300 python -u tools/ablate.py "$C" "$N" "${R:-5}" > "$OUT/ab_$C.txt" 2>&1 \
    || { tail -20 "$OUT/ab_$C.txt"; exit 1; }
  cat "$OUT/ab_$C.txt"
done
if [ "${3:-}" = "stamps" ]; then
  shift 3
  bash tools/gpu_stamps.sh "$TAG" "$@"
fi
