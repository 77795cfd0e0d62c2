#!/bin/bash
# Round-4 final library: the whole GPU test suite and smoke() (what the driver runs at round end).
set -e -o pipefail
OUT=gpurun_out/r04z
mkdir -p $OUT
sha256sum repic-copy_amd/repic_amd/librepic_gc.so > $OUT/lib_sha256.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rfE \
  > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $OUT/smoke.log 2>&1 \
  || { tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
