#!/bin/bash
# C2 file-to-file, three runs (box-to-box and run-to-run variance of the host-bound CLI).
set -e -o pipefail
mkdir -p gpurun_out/r04f2
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/file_bench.py --config C2 --n_mg 10000 > gpurun_out/r04f2/f2f_C2_$i.json 2> gpurun_out/r04f2/f2f_C2_$i.err \
    || { tail -20 gpurun_out/r04f2/f2f_C2_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04f2/f2f_C2_$i.json'));print(round(d['value']), d['wall_s'], d['phases_s'])"
done
