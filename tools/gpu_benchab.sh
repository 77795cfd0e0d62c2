#!/bin/bash
# The C2 headline (submit / wait path, 3 steps in flight) of abl/librepic_gc_zprev.so and of the
# working tree's library, alternated in fresh processes (REPIC_GC_LIB), after the submit-path
# GPU tests.
#   gpurun --timeout 900 -- bash tools/gpu_benchab.sh TAG [ROUNDS]
set -e -o pipefail
OUT=gpurun_out/${1:-benchab}; R=${2:-3}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "submit or lazy or cli or result_views or pipelined" > $OUT/pytest.log 2>&1 || { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; exit 1; }
tail -1 $OUT/pytest.log
for r in $(seq 1 $R); do
  for lib in abl/librepic_gc_zprev.so repic-copy_amd/repic_amd/librepic_gc.so; do
    n=$(basename $lib .so)
    REPIC_GC_LIB=$PWD/$lib timeout -k 10 200 python3 -u bench.py --by-config none --no-variants --no-cpu-baseline --steps 50 --warmup 10 > $OUT/b_${n}_$r.json 2> $OUT/b_${n}_$r.err || { tail -20 $OUT/b_${n}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${n}_$r.json')); print('$n', $r, round(d['value']), round(d['ms_per_step'], 4))"
  done
done
