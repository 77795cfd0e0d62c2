#!/bin/bash
# Round-4 final library evidence: rocprofv3 --kernel-trace --stats, PMC passes (traffic) and
# the bench line with its CPU baseline per config (tools/gpu_evidence.sh), then optionally the
# driver's default bench command (C2 headline + by_config), which reads the traffic JSONs the
# earlier calls left under profiles/.
#   gpurun -- bash tools/gpu_r04_final_evidence.sh "C2 C4" [default]
set -e -o pipefail
bash tools/gpu_evidence.sh r04z "$1"
if [ "${2:-}" = default ]; then
  timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 30 --warmup 10 > gpurun_out/r04z/bench_default.json \
    2> gpurun_out/r04z/bench_default.err || { tail -30 gpurun_out/r04z/bench_default.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04z/bench_default.json'));print(round(d['value']),d['ms_per_step'],d['roofline']['frac'],d['roofline']['bound']);[print(c,round(e['value']),e['ms_per_step'],e['roofline']['frac'],e['roofline']['bound']) for c,e in d.get('by_config',{}).items()]"
fi
