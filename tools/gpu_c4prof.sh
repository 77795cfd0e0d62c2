#!/bin/bash
# C4 phase profile: selected parity tests, interleaved ablation timing, per-phase stamps.
#   gpurun --timeout 600 -- bash tools/gpu_c4prof.sh TAG "pytest -k expr"
set -e -o pipefail
TAG=${1:-c4prof}; KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 200 python -u tools/ablate.py C4 4000 5 > "$OUT/ablate_c4.txt" 2>&1
cat "$OUT/ablate_c4.txt"
REPIC_GC_LIB=repic-copy_amd/repic_amd/librepic_gc_diag.so timeout -k 10 200 \
  python -u tools/phase_stamps.py C4 4000 > "$OUT/stamps_c4.txt" 2>&1
cat "$OUT/stamps_c4.txt"
