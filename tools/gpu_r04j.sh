#!/bin/bash
# r04j: contended output-reservation atomics (NORESV experiment) A/B on C2 / C4; ILP C5 timing.
set -e -o pipefail
mkdir -p gpurun_out/r04j
for C in "C2 10000 9" "C4 12500 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04j/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04j/ab_$1.txt; exit 1; }
  cat gpurun_out/r04j/ab_$1.txt
done
timeout -k 10 300 python -u -m pytest tests/test_ilp.py -m gpu -q --timeout 250 --timeout-method thread \
  -k full_c5 -s > gpurun_out/r04j/ilp_c5.log 2>&1 || { tail -30 gpurun_out/r04j/ilp_c5.log; exit 1; }
grep -E "full|ILP|passed|failed" gpurun_out/r04j/ilp_c5.log
