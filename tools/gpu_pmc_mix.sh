#!/bin/bash
# VALU instruction mix and SIMT lane efficiency of k_fused (one rocprofv3 pass per group).
#   gpurun --timeout 600 -- bash tools/gpu_pmc_mix.sh TAG [CONFIG] [N_MG]
set -e -o pipefail
TAG=${1:-mix}; CFG=${2:-C2}; NMG=${3:-10000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --config "$CFG" --n_mg "$NMG")
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    "${BENCH[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  find "$OUT/$name" -name '*counter_collection.csv' -exec cp {} "$OUT/$name.csv" \;
  python3 tools/pmc_summary.py k_fused "$OUT/$name.csv" | tee "$OUT/$name.txt"
}
pass mixa SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64
pass mixb SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_ATOMIC
echo "== done"
