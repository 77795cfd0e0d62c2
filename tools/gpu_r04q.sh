#!/bin/bash
# r04q: kernel + copy timeline of the C2 bench steps (gaps between launches), the ILP tests
# with the work-scaled node budget, then the file-to-file CLI per config.
set -e -o pipefail
OUT=gpurun_out/r04q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tl -o run -- \
  python3 bench.py --steps 20 --warmup 5 --by-config none --no-cpu-baseline > $OUT/tl_bench.json 2> $OUT/tl.err \
  || { tail -20 $OUT/tl.err; exit 1; }
find $OUT/tl -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/tl -name '*memory_copy_trace.csv' -exec cp {} $OUT/copy_trace.csv \; || true
timeout -k 10 600 python -u -m pytest tests/test_ilp.py -m gpu -q --timeout 400 --timeout-method thread \
  -k "full_c5 or default_limit or golden or synthetic" -rA -s > $OUT/ilp.log 2>&1 || { tail -40 $OUT/ilp.log; exit 1; }
grep -E "C3|full|ILP|inexact|passed|failed" $OUT/ilp.log | tail -12
for C in "C2 10000 300" "C3 4000 300" "C4 12500 400" "C5 64 600"; do
  set -- $C
  timeout -k 10 $3 python -u tools/file_bench.py --config $1 --n_mg $2 > $OUT/f2f_$1.json 2> $OUT/f2f_$1.err \
    || { tail -20 $OUT/f2f_$1.err; exit 1; }
  cat $OUT/f2f_$1.json
done
