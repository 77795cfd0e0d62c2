#!/bin/bash
# Round check: all GPU tests, smoke, the C2 bench line, rocprofv3 stats + kernel trace of the
# same command, then the C3/C4/C5 bench lines.  First failure ends the script.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG
set -e -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { grep -E "^E |FAILED|Error" "$OUT/pytest_gpu.log" | head -40; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('C2', round(d['value']), round(d['ms_per_step'],4), d['pipeline']['kernel_ms'], round(d['roofline']['frac'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/prof.err" || { tail -30 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/prof" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
head -6 "$OUT/kernel_stats.csv"
for C in C4 C3 C5; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps 10 --warmup 3 \
    > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || { tail -20 "$OUT/bench_$C.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));r=d['roofline'];print('$C', round(d['value']), round(d['ms_per_step'],4), round(r['frac'],4), r['kernel'][:30])"
done
