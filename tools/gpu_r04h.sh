#!/bin/bash
# r04h: P2 slow-box list A/B (abl/ variants) on C2 / C4, then fused-path parity tests.
set -e -o pipefail
mkdir -p gpurun_out/r04h
for C in "C2 10000 9" "C4 12500 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04h/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04h/ab_$1.txt; exit 1; }
  cat gpurun_out/r04h/ab_$1.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread \
  -x > gpurun_out/r04h/pytest.log 2>&1 || { tail -40 gpurun_out/r04h/pytest.log; exit 1; }
tail -3 gpurun_out/r04h/pytest.log
