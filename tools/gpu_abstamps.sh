#!/bin/bash
# Full GPU parity suite, interleaved A/B timing (ablate/ libraries vs the product build) and
# per-phase stamps of the diagnostic build, on C2 and C4.  First failure ends the script.
#   gpurun --timeout 900 -- bash tools/gpu_abstamps.sh TAG
set -e -o pipefail
TAG=${1:-abstamps}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for cn in C2:10000 C4:4000; do
  C=${cn%%:*}; N=${cn##*:}
  timeout -k 10 200 python -u tools/ablate.py $C $N 7 > "$OUT/ab_$C.txt" 2>&1 || { tail -20 "$OUT/ab_$C.txt"; exit 1; }
  cat "$OUT/ab_$C.txt"
  REPIC_GC_LIB=repic-copy_amd/repic_amd/librepic_gc_diag.so timeout -k 10 200 \
    python -u tools/phase_stamps.py $C $N > "$OUT/stamps_$C.txt" 2>&1 || { tail -20 "$OUT/stamps_$C.txt"; exit 1; }
  cat "$OUT/stamps_$C.txt"
done
