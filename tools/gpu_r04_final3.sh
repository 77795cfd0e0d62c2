#!/bin/bash
# Final library, call 3: single-config evidence (rocprof stats, PMC, bench + CPU baseline) for
# C2 and C5.
set -e -o pipefail
mkdir -p gpurun_out/r04z
sha256sum repic-copy_amd/repic_amd/librepic_gc.so > gpurun_out/r04z/lib_sha256_ev.txt
bash tools/gpu_evidence.sh r04z "C2 C5"
