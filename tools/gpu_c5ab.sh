#!/bin/bash
# Large-route check: its parity tests, then the C5 bench line with per-kernel times.
#   gpurun --timeout 900 -- bash tools/gpu_c5ab.sh TAG
set -e -o pipefail
OUT=gpurun_out/${1:-c5ab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "multikernel or dense_clusters or large_route or c5 or full_size or mixed" > $OUT/pytest.log 2>&1 \
  || { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --config C5 --by-config C5_256 --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c5.json'))
print('C5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms_per_step'])
print(d['pipeline']['kernel_ms'])
b=d['by_config']['C5_256']; print('C5_256', b['value'], b['ms_per_step'], b['roofline']['frac'], b['kernel_ms'])"
