#!/bin/bash
# r04u: BFS membership search from split A/B on C2 / C4; GPU
# parity + bench-step tests; phase stamps.
set -e -o pipefail
mkdir -p gpurun_out/r04u
for C in "C2 10000 9" "C4 12500 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04u/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04u/ab_$1.txt; exit 1; }
  cat gpurun_out/r04u/ab_$1.txt
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_threshold.py tests/test_distributed.py tests/test_bench_host.py -m gpu -q --timeout 300 --timeout-method thread \
  -x > gpurun_out/r04u/pytest.log 2>&1 || { tail -40 gpurun_out/r04u/pytest.log; exit 1; }
tail -2 gpurun_out/r04u/pytest.log
