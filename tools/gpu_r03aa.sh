set -e -o pipefail
bash tools/gpu_step.sh r03aa_t "multikernel or C5 or bench_step or large or golden or dense or k8"
bash tools/gpu_xp.sh r03aa "C5"
