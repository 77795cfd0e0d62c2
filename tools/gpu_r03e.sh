set -e -o pipefail
bash tools/gpu_xp.sh r03e "C2 C4"
bash tools/gpu_step.sh r03e_t "ilp or full_size or bench_step or dense or golden_and_not_multikernel" f2f pcs
