#!/bin/bash
# One iteration: A/B timing of ablate/*.so vs the product build on the given configs, then the
# GPU parity tests (except the ILP/score suites, whose kernels an A/B of k_fused leaves alone).
#   gpurun --timeout 900 -- bash tools/gpu_abt.sh TAG "C2 C4" ["PYTEST -k EXPR"]
set -e -o pipefail
TAG=${1:-abt}; CFGS=${2:-"C2 C4"}; KEXPR=${3:-"not ilp and not score"}
bash tools/gpu_xp.sh "$TAG" "$CFGS"
bash tools/gpu_step.sh "${TAG}_t" "$KEXPR"
