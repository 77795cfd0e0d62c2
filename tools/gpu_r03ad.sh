set -e -o pipefail
bash tools/gpu_xp.sh r03ad "C5"
bash tools/gpu_step.sh r03ad_t "multikernel or C5 or large or golden or k8"
