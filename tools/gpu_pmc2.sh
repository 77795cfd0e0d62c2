#!/bin/bash
# Occupancy + LDS PMC passes for one config, plus the SQ issue/stall
# passes and HBM traffic, and per-phase stamps from the diagnostic build.  Counters the
# device does not list are dropped from a pass (checked against `rocprofv3 -L` first).
#   gpurun --timeout 900 -- bash tools/gpu_pmc2.sh TAG CONFIG N_MG
set -e -o pipefail
TAG=${1:-pmc2}; CFG=${2:-C2}; NMG=${3:-10000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ ! -s "$OUT/../counters_avail.txt" ]; then
  timeout -s KILL 60 rocprofv3 -L > "$OUT/../counters_avail.txt" 2>&1 || true
fi
BENCH=(python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --config "$CFG" --n_mg "$NMG")
pass() {  # name counters...
  local name=$1
  shift
  local keep=()
  for c in "$@"; do
    if grep -q "\b$c\b" "$OUT/../counters_avail.txt"; then keep+=("$c"); else echo "  (no $c)"; fi
  done
  echo "== pass $name: ${keep[*]}"
  timeout -s KILL 90 rocprofv3 --pmc "${keep[@]}" --output-format csv -d "$OUT/$name" -o run -- \
    "${BENCH[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  find "$OUT/$name" -name '*counter_collection.csv' -exec cp {} "$OUT/$name.csv" \;
  python3 tools/pmc_summary.py k_fused "$OUT/$name.csv" | tee "$OUT/$name.txt"
}
pass occ SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
pass lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT
pass sqb SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 tools/pmc_traffic.py "$OUT/fetch.csv" "$OUT/write.csv" repic-copy_amd/repic_amd/librepic_gc.so "$OUT/traffic.json" "$CFG"
REPIC_GC_LIB=abl/librepic_gc_diag.so timeout -k 10 200 \
  python -u tools/phase_stamps.py "$CFG" "$NMG" > "$OUT/stamps.txt" 2>&1 || { tail -20 "$OUT/stamps.txt"; exit 1; }
cat "$OUT/stamps.txt"
echo "== done"
