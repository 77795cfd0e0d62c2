#!/bin/bash
# Occupancy sensitivity: fused kernel time at capped workgroups per CU (RGC_DIAG_MAX_WG).
#   gpurun --timeout 600 -- bash tools/gpu_occ.sh TAG
set -e -o pipefail
TAG=${1:-occ}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # config wgcap
  local C=$1 W=$2
  RGC_DIAG_MAX_WG=$W timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --steps 20 --warmup 5 \
    > "$OUT/b_${C}_$W.json" 2> "$OUT/b_${C}_$W.err" || { tail -20 "$OUT/b_${C}_$W.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b_${C}_$W.json'));print('$C wg<=$W', round(d['value']), d['pipeline']['kernel_ms'])"
}
run C2 128; run C2 3; run C2 2; run C2 128
run C4 128; run C4 1; run C4 128
