#!/bin/bash
# Bench lines for the other BASELINE configs (C3 crowded k=4, C4 k=5, C5 dense k=8).
#   gpurun --timeout 600 -- bash tools/gpu_configs.sh TAG
set -e -o pipefail
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for C in C4 C3 C5; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps 5 --warmup 2 \
    > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || { tail -20 "$OUT/bench_$C.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print('$C', d['value'], 'mg/s', d['ms_per_step'], 'ms/step', d['pipeline']['kernel_ms'], d['config']['micrographs_per_gpu'])"
done
