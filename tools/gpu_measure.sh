#!/bin/bash
# Measurement pass: default bench line (C2 + 1-core and parallel CPU baselines), the other
# configs, and the file-to-file CLI (C2 10k micrographs; 100k tiny micrographs).
#   gpurun --timeout 900 -- bash tools/gpu_measure.sh TAG
set -e -o pipefail
TAG=${1:-measure}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
for C in C3 C4 C5; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps 10 --warmup 3 \
    > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || { tail -20 "$OUT/bench_$C.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));r=d['roofline'];print('$C', round(d['value']), 'mg/s', round(r['frac'],4), r['kernel'])"
done
timeout -k 10 400 python -u tools/file_bench.py --config C2 --n_mg 10000 > "$OUT/f2f_c2.json" 2> "$OUT/f2f_c2.err" || { tail -20 "$OUT/f2f_c2.err"; exit 1; }
cat "$OUT/f2f_c2.json"
timeout -k 10 400 python -u tools/file_bench.py --config C2 --tiny --n_mg 100000 > "$OUT/f2f_tiny100k.json" 2> "$OUT/f2f_tiny100k.err" || { tail -20 "$OUT/f2f_tiny100k.err"; exit 1; }
cat "$OUT/f2f_tiny100k.json"
