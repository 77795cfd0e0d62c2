set -e -o pipefail
bash tools/gpu_xp.sh r03r "C2 C4" "384"
bash tools/gpu_step.sh r03r_t "not ilp and not score"
