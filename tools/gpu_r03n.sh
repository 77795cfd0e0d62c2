#!/bin/bash
# A/B + parity tests, then the file-to-file CLI with 1 / 4 / 16 native writer threads and the
# file-creation rate of the box's temp directory.
set -e -o pipefail
bash tools/gpu_abt.sh r03n "C2 C4"
OUT=gpurun_out/r03n_f2f
mkdir -p $OUT
for T in 4 1 16; do
  RGC_WRITER_THREADS=$T timeout -k 10 300 python -u tools/file_bench.py --config C2 --n_mg 10000 > $OUT/f2f_w$T.json 2> $OUT/f2f_w$T.err || { tail -20 $OUT/f2f_w$T.err; exit 1; }
  cat $OUT/f2f_w$T.json
done
timeout -k 10 120 python tools/fs_create_bench.py 20000 > $OUT/fs_create.json && cat $OUT/fs_create.json
