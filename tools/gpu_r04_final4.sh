#!/bin/bash
# Final library, call 4: single-config evidence for C4 and C3, then the driver's default bench
# line (C2 + by_config), which reads the traffic JSONs under profiles/.
set -e -o pipefail
bash tools/gpu_r04_final_evidence.sh "C4 C3" default
