set -e -o pipefail
OUT=gpurun_out/r03ai; mkdir -p $OUT
timeout -k 10 200 python -u tools/ablate_kernels.py C5 16 7 > $OUT/k16.txt 2>&1 || { tail $OUT/k16.txt; exit 1; }
cat $OUT/k16.txt
timeout -k 10 300 python -u tools/ablate_kernels.py C5 64 5 > $OUT/k64.txt 2>&1 || { tail $OUT/k64.txt; exit 1; }
cat $OUT/k64.txt
