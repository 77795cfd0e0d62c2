#!/bin/bash
# All GPU tests, smoke, then the default bench line (the driver's command).  First failure
# ends the script.
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh TAG
set -e -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --durations=10 > "$OUT/pytest_gpu.log" 2>&1 || { grep -E "^E |FAILED|Error" "$OUT/pytest_gpu.log" | head -40; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("C2", round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["frac"], 4),
      "stats_copy", d.get("stats_copy_variant", {}).get("value"))
for k, v in d.get("by_config", {}).items():
    r = v.get("roofline", {})
    print(k, round(v["value"], 1), v.get("ms_per_step", v.get("wall_s")), r.get("frac"), r.get("traffic_source"))
PY
