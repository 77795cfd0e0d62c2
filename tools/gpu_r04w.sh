#!/bin/bash
# r04w: write groups split by clique count (Python side only; the library is unchanged):
# CLI tests, then file-to-file C5 / C3 / C4.
set -e -o pipefail
OUT=gpurun_out/r04w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "cli or golden" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in "C5 64 600" "C3 4000 300" "C4 12500 400"; do
  set -- $C
  timeout -k 10 $3 python -u tools/file_bench.py --config $1 --n_mg $2 > $OUT/f2f_$1.json 2> $OUT/f2f_$1.err \
    || { tail -20 $OUT/f2f_$1.err; exit 1; }
  cat $OUT/f2f_$1.json
done
