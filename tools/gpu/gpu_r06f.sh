#!/bin/bash
# r06: compact factor v4 A/B (LBA tests + batch bench) and then its PMC breakdown against the whole-Hpl form
set -o pipefail
bash tools/gpu/gpu_r06b.sh ${1:-r06f} && bash tools/gpu/gpu_r06e.sh ${2:-r06fp}
