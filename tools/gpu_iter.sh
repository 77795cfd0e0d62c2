#!/bin/bash
# Quick GPU iteration: parity tests, then ablation timings (per-phase marginal cost) and a
# short bench line.  First failure ends the script.
#   gpurun --timeout 600 -- bash tools/gpu_iter.sh TAG [CONFIG] [N_MG]
set -e -o pipefail
TAG=${1:-iter}; CFG=${2:-C2}; NMG=${3:-10000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { grep -E "^E |FAILED|Error" "$OUT/pytest_gpu.log" | head -30; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u tools/ablate.py "$CFG" "$NMG" 7 > "$OUT/ablate.txt" 2>&1 \
  || { tail -20 "$OUT/ablate.txt"; exit 1; }
cat "$OUT/ablate.txt"
timeout -k 10 200 python -u bench.py --config "$CFG" --n_mg "$NMG" --no-cpu-baseline \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['pipeline']['kernel_ms'])"
if [ -f repic-copy_amd/repic_amd/librepic_gc_diag.so ]; then
  timeout -k 10 200 python -u tools/phase_stamps.py "$CFG" "$NMG" > "$OUT/stamps.txt" 2>&1 \
    || { tail -20 "$OUT/stamps.txt"; exit 1; }
  cat "$OUT/stamps.txt"
fi
