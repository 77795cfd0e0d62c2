set -e -o pipefail
OUT=gpurun_out/r03aj; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/ablate_kernels.py C5 64 5 > $OUT/k64.txt 2>&1 || { tail $OUT/k64.txt; exit 1; }
cat $OUT/k64.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --config C5 --no-cpu-baseline --steps 6 --warmup 2 > "$OUT/bench_prof.json" 2> "$OUT/prof.err" || { tail -30 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
head -12 "$OUT/kernel_stats.csv" | cut -c1-120
