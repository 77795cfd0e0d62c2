#!/bin/bash
# Selected GPU tests (-k expression), then bench lines for the given configs.
#   gpurun --timeout 900 -- bash tools/gpu_quick.sh TAG "pytest -k expr" "C3 C5 ..."
set -e -o pipefail
TAG=${1:-quick}
KEXPR=${2:-}
CFGS=${3:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
for C in $CFGS; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps 10 --warmup 3 \
    > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || { tail -20 "$OUT/bench_$C.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print('$C', round(d['value']), 'mg/s', round(d['ms_per_step'],3), 'ms/step', d['pipeline']['kernel_ms'])"
done
