#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats.  Every GPU step has its
# own time limit; the first failure ends the script (no retries).
#   gpurun --timeout 1100 -- bash tools/gpu_check.sh [tag] [bench args...]
set -e -o pipefail
TAG=${1:-run}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "== smoke"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== rocprofv3 stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_prof.json" 2> "$OUT/prof.err" \
  || { tail -30 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
head -12 "$OUT/kernel_stats.csv"
echo "== done"
