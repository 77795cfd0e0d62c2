#!/bin/bash
# r04x: fractional-coordinate micrographs (f64 layout) vs integer ones on C2 / C4.
set -e -o pipefail
mkdir -p gpurun_out/r04x
for C in "C2 10000" "C4 12500"; do
  set -- $C
  timeout -k 10 300 python -u tools/frac_bench.py $1 $2 5 > gpurun_out/r04x/frac_$1.json 2> gpurun_out/r04x/frac_$1.err || { tail -20 gpurun_out/r04x/frac_$1.err; exit 1; }
  cat gpurun_out/r04x/frac_$1.json
done
