#!/bin/bash
# Per-kernel durations (rocprofv3 kernel-trace stats) of a short serialised bench run.
#   gpurun --timeout 600 -- bash tools/gpu_ks.sh TAG CONFIG [N_MG]
set -e -o pipefail
TAG=${1:-ks}; CFG=${2:-C5}; NMG=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
ARGS=(--no-cpu-baseline --by-config none --streams 1 --no-variants --steps 10 --warmup 2 --config $CFG)
if [ -n "$NMG" ]; then ARGS+=(--n_mg $NMG); fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_$CFG -o run -- python3 bench.py "${ARGS[@]}" > $OUT/ks_$CFG.json 2> $OUT/ks_$CFG.err || { tail -20 $OUT/ks_$CFG.err; exit 1; }
find $OUT/ks_$CFG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$CFG.csv \;
python3 - "$OUT/kernel_stats_$CFG.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print("%-60s calls %6s avg %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
