set -e -o pipefail
OUT=gpurun_out/r03ab; mkdir -p $OUT
for E in 0 1; do
  if [ $E = 1 ]; then export RGC_NO_LEAF_EPI=1; fi
  timeout -k 10 200 python -u bench.py --config C5 --no-cpu-baseline --steps 8 --warmup 2 > $OUT/c5_noleaf$E.json 2> $OUT/c5_noleaf$E.err
  python3 -c "import json;d=json.load(open('$OUT/c5_noleaf$E.json'));print('NO_LEAF_EPI=$E', round(d['value']), d['pipeline']['kernel_ms'])"
done
