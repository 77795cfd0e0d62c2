set -e -o pipefail
bash tools/gpu_xp.sh r03w "C5"
bash tools/gpu_step.sh r03w_t "multikernel or C5 or bench_step or large or golden"
