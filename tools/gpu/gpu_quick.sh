#!/bin/bash
# Matcher + pose parity tests and the single-call latency probe with phase clocks (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03quick}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_match_gpu.py tests/test_ba_gpu.py tests/test_golden_ba.py tests/test_adapter.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
OSG_MATCH_PROFILE=1 timeout -k 10 120 python3 tools/latency_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err
echo "pytest=$rc probe=$?"
