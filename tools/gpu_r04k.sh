#!/bin/bash
# r04k: reservation atomic overlapped with P5 (product) vs no reservation (NORESV) vs r03 on
# C2 / C4; fused parity tests; ILP tests (wave search stops at Gurobi's MIPGap).
set -e -o pipefail
mkdir -p gpurun_out/r04k
for C in "C2 10000 9" "C4 12500 5"; do
  set -- $C
  timeout -k 10 300 python -u tools/ablate.py $1 $2 $3 > gpurun_out/r04k/ab_$1.txt 2>&1 || { tail -20 gpurun_out/r04k/ab_$1.txt; exit 1; }
  cat gpurun_out/r04k/ab_$1.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread \
  -x > gpurun_out/r04k/pytest.log 2>&1 || { tail -40 gpurun_out/r04k/pytest.log; exit 1; }
tail -2 gpurun_out/r04k/pytest.log
timeout -k 10 600 python -u -m pytest tests/test_ilp.py -m gpu -q --timeout 400 --timeout-method thread \
  -rA -s > gpurun_out/r04k/ilp.log 2>&1 || { tail -60 gpurun_out/r04k/ilp.log; exit 1; }
grep -E "C3|C5|full|ILP|inexact|passed|failed" gpurun_out/r04k/ilp.log | tail -30
