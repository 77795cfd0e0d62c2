#!/bin/bash
# Fused-kernel change: the parity tests that run the fused route, then interleaved A/B of
# abl/*.so against the working tree's library on C2, C4, C3 (tools/ablate.py).
#   gpurun --timeout 900 -- bash tools/gpu_abfused.sh TAG
set -e -o pipefail
OUT=gpurun_out/${1:-abf}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_threshold.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; exit 1; }
tail -1 $OUT/pytest.log
for cn in C2:10000 C4:12500 C3:4000; do
  C=${cn%%:*}; N=${cn##*:}
  timeout -k 10 300 python -u tools/ablate.py $C $N 9 > $OUT/ab_$C.txt 2>&1 || { tail -5 $OUT/ab_$C.txt; exit 1; }
  cat $OUT/ab_$C.txt
done
