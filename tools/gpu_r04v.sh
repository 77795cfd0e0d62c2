#!/bin/bash
# r04v: large-route variants (k2_pairs register fill; + segmented leaf marks) A/B on C5 / C3,
# then the large-route parity tests on the combined variant (REPIC_GC_LIB).
set -e -o pipefail
mkdir -p gpurun_out/r04v
for C in "C5 64 5" "C3 4000 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04v/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04v/ab_$1.txt; exit 1; }
  cat gpurun_out/r04v/ab_$1.txt
done
REPIC_GC_LIB=abl/librepic_gc_zk2lm.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_threshold.py -m gpu -q --timeout 300 --timeout-method thread \
  -x > gpurun_out/r04v/pytest.log 2>&1 || { tail -40 gpurun_out/r04v/pytest.log; exit 1; }
tail -2 gpurun_out/r04v/pytest.log
