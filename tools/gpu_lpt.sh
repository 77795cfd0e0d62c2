set -e -o pipefail
OUT=gpurun_out/r03z; mkdir -p $OUT
for i in 1 2; do for L in 0 1; do
  RGC_LPT=$L timeout -k 10 200 python -u bench.py --config C2 --no-cpu-baseline --steps 30 --warmup 5 > $OUT/c2_lpt$L.json 2> $OUT/c2_lpt$L.err
  python3 -c "import json;d=json.load(open('$OUT/c2_lpt$L.json'));r=d['roofline'];print('C2 LPT=$L', round(d['value']), round(d['ms_per_step'],4), round(r['kernel_ms_per_step'],4))"
  RGC_LPT=$L timeout -k 10 200 python -u bench.py --config C4 --no-cpu-baseline --steps 30 --warmup 5 > $OUT/c4_lpt$L.json 2> $OUT/c4_lpt$L.err
  python3 -c "import json;d=json.load(open('$OUT/c4_lpt$L.json'));r=d['roofline'];print('C4 LPT=$L', round(d['value']), round(d['ms_per_step'],4), round(r['kernel_ms_per_step'],4))"
done; done
