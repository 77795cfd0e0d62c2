#!/bin/bash
# Timing-only GPU pass: every library under abl/ plus the product build, timed
# interleaved in one process (tools/ablate.py).  No parity tests: experiments only.
#   gpurun --timeout 300 -- bash tools/gpu_ab.sh TAG [CONFIG] [N_MG]
set -e -o pipefail
TAG=${1:-ab}; CFG=${2:-C2}; NMG=${3:-10000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 200 python -u tools/ablate.py "$CFG" "$NMG" 7 > "$OUT/ablate.txt" 2>&1 \
  || { tail -20 "$OUT/ablate.txt"; exit 1; }
cat "$OUT/ablate.txt"
