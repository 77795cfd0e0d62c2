#!/bin/bash
# Selected GPU tests (-k expression, optional), then the driver's default bench command (C2
# headline + by_config C3/C4/C5) with its CPU baseline.
#   gpurun --timeout 900 -- bash tools/gpu_bench_byconfig.sh TAG ["pytest -k expr"]
set -e -o pipefail
TAG=${1:-bc}
KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("headline", d["config"]["workload"][:2], round(d["value"]), round(d["ms_per_step"], 4),
      round(d["roofline"]["frac"], 4), d["roofline"]["bound"])
for c, e in d.get("by_config", {}).items():
    print(c, round(e["value"]), round(e["ms_per_step"], 4), round(e["kernel_ms"], 4),
          round(e["roofline"]["frac"], 4), e["roofline"]["bound"])
PY
