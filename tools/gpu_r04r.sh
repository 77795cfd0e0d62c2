#!/bin/bash
# r04r: step gaps with / without timing events; union variants A/B on C2 / C4.
set -e -o pipefail
mkdir -p gpurun_out/r04r
timeout -k 10 300 python -u tools/step_gap.py C2 10000 30 > gpurun_out/r04r/step_gap.json 2> gpurun_out/r04r/step_gap.err || { tail -20 gpurun_out/r04r/step_gap.err; exit 1; }
cat gpurun_out/r04r/step_gap.json
for C in "C2 10000 9" "C4 12500 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04r/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04r/ab_$1.txt; exit 1; }
  cat gpurun_out/r04r/ab_$1.txt
done
