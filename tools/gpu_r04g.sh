#!/bin/bash
# r04g: A/B of the P1 grid plan by wave 0 vs every wave (abl/ variants) on C2 / C4.
set -e -o pipefail
mkdir -p gpurun_out/r04g
for C in "C2 10000 9" "C4 12500 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04g/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04g/ab_$1.txt; exit 1; }
  cat gpurun_out/r04g/ab_$1.txt
done
