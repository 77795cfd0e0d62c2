#!/bin/bash
# Per-phase PMC attribution: each ablation build (fused kernel stops after phase N) and the
# product build run under one SQ counter pass; marginal counts per phase = differences.
#   make -C repic-copy_amd/csrc ablate && gpurun --timeout 900 -- bash tools/gpu_pmc_ablate.sh TAG [C2] [n_mg] [COUNTERS]
# COUNTERS (one pass, <= 8 SQ counters): default the issue/stall set; "lane" = VALU lane
# efficiency per phase (SQ_ACTIVE_INST_VALU, SQ_THREAD_CYCLES_VALU, SQ_INSTS_VALU).
# LIBS (glob, default abl/librepic_gc_stop*.so): the libraries measured before the product
set -e -o pipefail
TAG=${1:-pmcabl}; CFG=${2:-C2}; NMG=${3:-10000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CNT=${4:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"}
[ "$CNT" = lane ] && CNT="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"
LIBS=${LIBS:-"abl/librepic_gc_stop*.so"}
for L in $LIBS repic-copy_amd/repic_amd/librepic_gc.so; do
  b=$(basename "$L" .so)
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/$b" -o run -- \
    python3 tools/ablate.py "$CFG" "$NMG" 1 "$L" > "$OUT/$b.txt" 2> "$OUT/$b.err" || { tail -20 "$OUT/$b.err"; exit 1; }
  find "$OUT/$b" -name '*counter_collection.csv' -exec cp {} "$OUT/$b.csv" \;
  echo "== $b" | tee -a "$OUT/summary.log"
  python3 tools/pmc_summary.py "k_fused<" "$OUT/$b.csv" | tee -a "$OUT/summary.log"
done
python3 tools/pmc_ablate_delta.py "$OUT/summary.log" | tee "$OUT/delta.txt"
echo "== done"
