#!/bin/bash
# k_pose_lat: pose parity tests (every variant) and the single-call latency probe (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03poselat}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pose" > $OUT/pytest.log 2>&1
rc=$?
timeout -k 10 120 python3 tools/latency_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err
echo "pytest=$rc probe=$?"
