#!/bin/bash
# C5 route: HBM traffic per step (FETCH_SIZE / WRITE_SIZE passes) of a short serialised bench.
set -e -o pipefail
OUT=gpurun_out/${1:-c5pmc}; mkdir -p $OUT
export TMPDIR=/tmp
B=(python3 bench.py --config C5 --no-cpu-baseline --by-config none --streams 1 --no-variants --steps 3 --warmup 1)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- "${B[@]}" > $OUT/$c.json 2> $OUT/$c.err || { tail -5 $OUT/$c.err; exit 1; }
  find $OUT/$c -name '*counter_collection.csv' -exec cp {} $OUT/$c.csv \;
done
python3 - $OUT <<'PY'
import csv, sys, collections
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    tot = collections.Counter()
    for r in csv.DictReader(open(f"{out}/{c}.csv")):
        tot[r["Kernel_Name"].split("(")[0][:40]] += float(r["Counter_Value"])
    s = sum(tot.values())
    print(c, f"{s * 1024 / 4 / 1e9:.2f} GB per step (4 steps)", [(k, round(v * 1024 / 4 / 1e6)) for k, v in tot.most_common(6)])
PY
