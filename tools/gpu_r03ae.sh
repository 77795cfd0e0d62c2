set -e -o pipefail
OUT=gpurun_out/r03ae; mkdir -p $OUT
RGC_DIAG_EXCOUNT=1 timeout -k 10 200 python -u bench.py --config C5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err
grep "rgc diag" $OUT/c5.err | sort | uniq -c | head -5
bash tools/gpu_xp.sh r03ae "C5"
