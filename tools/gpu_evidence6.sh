#!/bin/bash
# Evidence per by_config entry (round 6): rocprofv3 --kernel-trace --stats of the entry's bench
# with its steps serialised on one stream (--streams 1: per-launch durations that do not
# overlap, as the line's roofline leg times them), then the PMC passes whose traffic /
# counters bench.py folds into that entry's roofline (tools/gpu_pmc.sh, record keyed by entry).
#   gpurun --timeout 1200 -- bash tools/gpu_evidence6.sh TAG "C2:C2:10000 C4_100k:C4:100000 ..."
set -e -o pipefail
TAG=${1:-ev}; ITEMS=${2:-"C2:C2:10000"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for it in $ITEMS; do
  E=${it%%:*}; rest=${it#*:}; C=${rest%%:*}; N=${rest#*:}
  echo "== $E ($C, $N micrographs) stats"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$E" -o run -- \
    python3 bench.py --config $C --n_mg $N --no-cpu-baseline --by-config none --streams 1 --no-variants \
    > "$OUT/bench_prof_$E.json" 2> "$OUT/prof_$E.err" || { tail -30 "$OUT/prof_$E.err"; exit 1; }
  find "$OUT/prof_$E" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$E.csv" \;
  head -4 "$OUT/kernel_stats_$E.csv"
  echo "== $E pmc"
  bash tools/gpu_pmc.sh "$TAG/pmc_$E" "$C" "$N" "$E" > "$OUT/pmc_$E.log" 2>&1 || { tail -30 "$OUT/pmc_$E.log"; exit 1; }
  tail -2 "$OUT/pmc_$E.log"
done
