#!/bin/bash
# VALU cycle calibration: tools/probe/valu_cal (built on the CPU side,
# `hipcc --offload-arch=gfx950 -O3 -o tools/probe/valu_cal tools/probe/valu_cal.hip`) timed
# plain, then one rocprofv3 PMC pass per counter group.  Output under gpurun_out/TAG.
#   gpurun --timeout 300 -- bash tools/gpu_valu_cal.sh TAG
set -e -o pipefail
TAG=${1:-valucal}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/valu_cal > "$OUT/plain.json"
pass() {
  local name=$1
  shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    ./tools/probe/valu_cal > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  find "$OUT/$name" -name '*counter_collection.csv' -exec cp {} "$OUT/$name.csv" \;
}
pass a SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
pass b SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAVES GRBM_COUNT
echo "== done"
