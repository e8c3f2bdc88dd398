#!/bin/bash
# r06: the compact-factor Schur A/B (tools/gpu/gpu_r06b.sh) and the FP4 top-2 skip-test A/B (gpu_r06c.sh) in one call
set -o pipefail
bash tools/gpu/gpu_r06b.sh ${1:-r06b} && bash tools/gpu/gpu_r06c.sh ${2:-r06c}
