#!/bin/bash
# PMC passes over a short bench run of one config: SQ issue/stall counters, VALU lane cycles,
# HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes, per MI355X_MICROARCH.md), GRBM
# clock.  One counter group per rocprofv3 run, each under its own SIGKILL time limit; the first
# failure ends the script.  tools/pmc_traffic.py folds them into OUT/traffic.json (bench.py
# reads it from profiles/ when the library sha256 and the config match).
#   gpurun --timeout 900 -- bash tools/gpu_pmc.sh TAG [CONFIG] [N_MG] [ENTRY]
# ENTRY: the bench.py by_config name the counters stand for (default CONFIG; e.g. C4 100000
# C4_100k): bench.py matches records by entry, so each batch size has its own.
set -e -o pipefail
TAG=${1:-pmc}; CFG=${2:-C2}; NMG=${3:-}; ENTRY=${4:-$CFG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=3; WARM=1
BENCH=(python3 bench.py --no-cpu-baseline --by-config none --streams 1 --no-variants --steps $STEPS --warmup $WARM --config "$CFG")
if [ -n "$NMG" ]; then BENCH+=(--n_mg "$NMG"); fi
KSUB="k_fused<"
if [ "$CFG" = "C5" ]; then KSUB=rgc::; fi
pass() {  # name counters...
  local name=$1
  shift
  echo "== pass $name: $*"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    "${BENCH[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  find "$OUT/$name" -name '*counter_collection.csv' -exec cp {} "$OUT/$name.csv" \;
  python3 tools/pmc_summary.py "$KSUB" "$OUT/$name.csv"
}
pass sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS
pass sqb SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH
pass lane SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 tools/pmc_traffic.py "$OUT" repic-copy_amd/repic_amd/librepic_gc.so "$OUT/traffic.json" "$CFG" $((STEPS + WARM)) "$ENTRY"
echo "== done"
