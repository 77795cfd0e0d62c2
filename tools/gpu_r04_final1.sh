#!/bin/bash
# Final library, call 1: the whole GPU suite + smoke, large-route A/B against the previous
# build (abl/), then the C2 evidence (rocprof stats, PMC, bench line with its CPU baseline).
set -e -o pipefail
OUT=gpurun_out/r04z
mkdir -p $OUT
sha256sum repic-copy_amd/repic_amd/librepic_gc.so > $OUT/lib_sha256.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rfE \
  > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $OUT/smoke.log 2>&1 \
  || { tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for C in "C5 64 5" "C3 4000 3"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > $OUT/ab_$1.txt 2>&1 || { tail -20 $OUT/ab_$1.txt; exit 1; }
  cat $OUT/ab_$1.txt
done
bash tools/gpu_evidence.sh r04z "C2"
