#!/bin/bash
# Large-route change: its parity tests, then interleaved A/B of abl/*.so against the working
# tree's library on C5 (64 and 256 micrographs per step, tools/ablate.py).
#   gpurun --timeout 900 -- bash tools/gpu_c5abl.sh TAG
set -e -o pipefail
OUT=gpurun_out/${1:-c5abl}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "multikernel or dense_clusters or large_route or c5 or full_size or mixed or synthetic" > $OUT/pytest.log 2>&1 \
  || { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; exit 1; }
tail -1 $OUT/pytest.log
for cn in C5:64 C5:256; do
  C=${cn%%:*}; N=${cn##*:}
  timeout -k 10 300 python -u tools/ablate.py $C $N 9 > $OUT/ab_${C}_$N.txt 2>&1 || { tail -5 $OUT/ab_${C}_$N.txt; exit 1; }
  cat $OUT/ab_${C}_$N.txt
done
