#!/bin/bash
# Latency probe with the matchers' phase clocks (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03probe}
mkdir -p $OUT
cd $R
OSG_MATCH_PROFILE=1 timeout -k 10 120 python3 tools/latency_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err
echo "probe=$?"
