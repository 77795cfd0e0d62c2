#!/bin/bash
# Measurement evidence per config: the bench line with its CPU baseline,
# rocprofv3 --kernel-trace --stats of the same bench with its steps serialised on one stream
# (--streams 1: per-launch durations that do not overlap, as the default line's roofline leg
# times them), and the PMC passes whose traffic / counters bench.py folds into roofline.traffic
# / limiter (tools/gpu_pmc.sh).
#   gpurun --timeout 1200 -- bash tools/gpu_evidence.sh TAG "C2 C3 C4 C5"
set -e -o pipefail
TAG=${1:-ev}; CFGS=${2:-"C2 C3 C4 C5"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in $CFGS; do
  echo "== $C stats"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$C" -o run -- \
    python3 bench.py --config $C --no-cpu-baseline --by-config none --streams 1 --no-variants > "$OUT/bench_prof_$C.json" 2> "$OUT/prof_$C.err" \
    || { tail -30 "$OUT/prof_$C.err"; exit 1; }
  find "$OUT/prof_$C" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$C.csv" \;
  head -8 "$OUT/kernel_stats_$C.csv"
  echo "== $C pmc"
  bash tools/gpu_pmc.sh "$TAG/pmc_$C" "$C" > "$OUT/pmc_$C.log" 2>&1 || { tail -30 "$OUT/pmc_$C.log"; exit 1; }
  tail -3 "$OUT/pmc_$C.log"
  # the bench line reads traffic from profiles/ (matched by library sha256 and config)
  cp "$OUT/pmc_$C/traffic.json" "profiles/${TAG}_${C,,}_traffic.json"
done
for C in $CFGS; do
  echo "== $C bench + cpu baseline"
  timeout -k 10 400 python3 -u bench.py --config $C --by-config none > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" \
    || { tail -30 "$OUT/bench_$C.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));r=d['roofline'];print('$C', round(d['value']), round(d['ms_per_step'],4), round(r['frac'],4), d.get('cpu_baseline',{}).get('value'))"
done
