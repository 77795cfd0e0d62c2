set -e -o pipefail
OUT=gpurun_out/r03ac; mkdir -p $OUT
bash tools/gpu_step.sh r03ac_t "multikernel or C5 or bench_step or large or golden or dense or k8"
bash tools/gpu_xp.sh r03ac "C5"
timeout -k 10 200 python -u bench.py --config C5 --no-cpu-baseline --steps 8 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print(round(d['value']), d['pipeline']['kernel_ms'])"
