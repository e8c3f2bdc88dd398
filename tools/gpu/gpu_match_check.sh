#!/bin/bash
# Matcher parity tests + single-call latency probe (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03match}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_match_gpu.py $R/tests/test_dbow_gpu.py $R/tests/test_adapter.py $R/tests/test_shard_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 &&
OSG_MATCH_PROFILE=1 timeout -k 10 120 python3 $R/tools/latency_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err &&
timeout -k 10 200 python3 $R/tools/match_batch_bench.py > $OUT/batch.jsonl 2> $OUT/batch.err
echo "exit=$?"
