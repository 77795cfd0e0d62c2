set -e -o pipefail
OUT=gpurun_out/r03af; mkdir -p $OUT
bash tools/gpu_step.sh r03af_t "multikernel or C5 or bench_step or large or golden or dense or k8 or multi"
bash tools/gpu_xp.sh r03af "C5"
timeout -k 10 200 python -u bench.py --config C5 --no-cpu-baseline --steps 8 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print(round(d['value']), d['roofline']['frac'], d['pipeline']['kernel_ms'])"
