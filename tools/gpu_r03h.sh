set -e -o pipefail
bash tools/gpu_xp.sh r03h "C2 C4"
bash tools/gpu_step.sh r03h_t "not ilp and not score"
