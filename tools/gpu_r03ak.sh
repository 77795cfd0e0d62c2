set -e -o pipefail
OUT=gpurun_out/r03ak; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_step.sh r03ak_t "multikernel or C5 or large or golden or k8 or dense or epilogue"
timeout -k 10 200 python -u tools/ablate_kernels.py C5 64 5 > $OUT/k64.txt 2>&1 || { tail $OUT/k64.txt; exit 1; }
cat $OUT/k64.txt
