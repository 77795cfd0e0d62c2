#!/bin/bash
# Chained GPU checks for one iteration: selected GPU tests, then optional file-to-file bench
# and PC sampling.  The first failing step ends the script.
#   gpurun --timeout 1100 -- bash tools/gpu_step.sh TAG "PYTEST -k EXPR" [f2f] [pcs]
set -e -o pipefail
TAG=${1:-step}; KEXPR=${2:-}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "$KEXPR" -s > "$OUT/pytest_gpu.log" 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" "$OUT/pytest_gpu.log" | tail -40; exit 1; }
  grep -E "passed|failed" "$OUT/pytest_gpu.log" | tail -2
  grep -E "status|gap" "$OUT/pytest_gpu.log" | head -20 || true
fi
for s in "$@"; do
  case $s in
    f2f)
      timeout -k 10 400 python -u tools/file_bench.py --config C2 --n_mg 10000 > "$OUT/f2f_c2.json" 2> "$OUT/f2f_c2.err" || { tail -20 "$OUT/f2f_c2.err"; exit 1; }
      cat "$OUT/f2f_c2.json" ;;
    pcs)
      bash tools/gpu_pcs.sh "$TAG/pcs" C2 host_trap time 1 ;;
  esac
done
