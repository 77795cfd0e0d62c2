#!/bin/bash
# A/B timing of abl/*.so against the product build on C2, C4 and C5 (tools/ablate.py,
# interleaved in one process per config).
set -e -o pipefail
TAG=${1:-ab3}
mkdir -p gpurun_out/$TAG
for C in "C2 10000 7" "C4 12500 5" "C5 64 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/$TAG/ab_$1.txt 2>&1 || { tail -20 gpurun_out/$TAG/ab_$1.txt; exit 1; }
  cat gpurun_out/$TAG/ab_$1.txt
done
