#!/bin/bash
# Final library, call 2: evidence for C4, C3, C5, then the driver's default bench line.
set -e -o pipefail
bash tools/gpu_r04_final_evidence.sh "C4 C3 C5" default
