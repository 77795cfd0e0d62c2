#!/bin/bash
# PC sampling (rocprofv3 beta) of a short bench run: where the fused kernel's issue time goes,
# instruction by instruction.  One method per run, each under its own SIGKILL limit.
#   gpurun --timeout 600 -- bash tools/gpu_pcs.sh TAG [CONFIG] [METHOD] [UNIT] [INTERVAL]
set -e -o pipefail
TAG=${1:-pcs}; CFG=${2:-C2}; METHOD=${3:-host_trap}; UNIT=${4:-time}; IV=${5:-1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method "$METHOD" \
  --pc-sampling-unit "$UNIT" --pc-sampling-interval "$IV" --output-format csv -d "$OUT/pcs" -o run -- \
  python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --config "$CFG" > "$OUT/bench.json" 2> "$OUT/pcs.err" \
  || { tail -30 "$OUT/pcs.err"; exit 1; }
find "$OUT/pcs" -type f | head -20
for f in $(find "$OUT/pcs" -name '*.csv'); do echo "== $f"; head -3 "$f"; wc -l "$f"; done
