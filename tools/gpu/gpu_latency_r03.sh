#!/bin/bash
# Single-call latency breakdown (one gpurun call): the probe with the matchers' in-kernel phase clocks,
# then under a HIP API + kernel + copy trace (no counters).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03lat}
mkdir -p $OUT
OSG_MATCH_PROFILE=1 timeout -k 10 120 python3 $R/tools/latency_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err &&
cd /tmp && timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace -o lat -- python3 $R/tools/latency_probe.py > $OUT/probe_traced.jsonl 2> $OUT/trace.err
echo "exit=$?"
