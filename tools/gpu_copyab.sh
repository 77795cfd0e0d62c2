#!/bin/bash
# The default line's stats-copy variant four times in fresh processes on one box (round 6:
# its per-micrograph stats copy as a blit packet read 14.3-14.8 M or 25 M micrographs/s by how
# the process's streams mapped onto hardware queues; RGC_BENCH_COPY, which chose the copy
# stream, is gone with that copy: the modes now run the same code).
#   gpurun --timeout 900 -- bash tools/gpu_copyab.sh TAG
set -e -o pipefail
OUT=gpurun_out/${1:-copyab}; mkdir -p $OUT
for r in 1 2; do
  for mode in null high; do
    RGC_BENCH_COPY=$mode timeout -k 10 200 python3 -u bench.py --by-config none --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b_${mode}_$r.json 2> $OUT/b_${mode}_$r.err || { tail -20 $OUT/b_${mode}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/b_${mode}_$r.json')); print('$mode', $r, round(d['value']), round(d['stats_copy_variant']['value']), round(d['stats_copy_variant']['ms_per_step'],4))"
  done
done
