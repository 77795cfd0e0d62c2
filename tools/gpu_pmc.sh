#!/bin/bash
# PMC passes over a short bench run: SQ issue/stall counters, HBM traffic (FETCH_SIZE and
# WRITE_SIZE in separate passes, per MI355X_MICROARCH.md), GRBM clock.  One counter group per
# rocprofv3 run, each under its own SIGKILL time limit; the first failure ends the script.
#   gpurun --timeout 900 -- bash tools/gpu_pmc.sh TAG [bench args...]
set -e -o pipefail
TAG=${1:-pmc}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@")
pass() {  # name counters...
  local name=$1
  shift
  echo "== pass $name: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    "${BENCH[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  find "$OUT/$name" -name '*counter_collection.csv' -exec cp {} "$OUT/$name.csv" \;
  python3 tools/pmc_summary.py k_fused "$OUT/$name.csv"
}
pass sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS
pass sqb SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 tools/pmc_traffic.py "$OUT/fetch.csv" "$OUT/write.csv" repic-copy_amd/repic_amd/librepic_gc.so "$OUT/traffic.json" "$(python3 -c 'import sys;a=sys.argv[1:];print(a[a.index("--config")+1] if "--config" in a else "C2")' "$@")"
echo "== done"
