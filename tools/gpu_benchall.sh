#!/bin/bash
# Bench lines of every config (no CPU baseline) after the GPU tests; first failure ends it.
#   gpurun --timeout 1100 -- bash tools/gpu_benchall.sh TAG ["PYTEST -k EXPR"]
set -e -o pipefail
TAG=${1:-benchall}; KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$KEXPR" ]; then bash tools/gpu_step.sh "${TAG}_t" "$KEXPR"; fi
for C in C2 C4 C3 C5; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps 20 --warmup 5 \
    > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || { tail -20 "$OUT/bench_$C.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));r=d['roofline'];print('$C', round(d['value']), round(d['ms_per_step'],4), round(r['kernel_ms_per_step'],4), round(r['frac'],4))"
done
