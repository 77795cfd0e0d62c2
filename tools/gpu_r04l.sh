#!/bin/bash
# r04l: batch-cursor atomics A/B (no reservation / no edge sum / 8 sharded cursors) on C2 / C4;
# per-phase s_memtime shares of the diagnostic build on C2.
set -e -o pipefail
mkdir -p gpurun_out/r04l
for C in "C2 10000 9" "C4 12500 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04l/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04l/ab_$1.txt; exit 1; }
  cat gpurun_out/r04l/ab_$1.txt
done
REPIC_GC_LIB=repic-copy_amd/repic_amd/librepic_gc_diag.so timeout -k 10 300 python -u tools/phase_stamps.py C2 10000 > gpurun_out/r04l/stamps_C2.txt 2>&1 || { tail -20 gpurun_out/r04l/stamps_C2.txt; exit 1; }
cat gpurun_out/r04l/stamps_C2.txt
