#!/bin/bash
# The adapter's in-place pose gather: the adapter GPU tests, then the C3 / C5 wall probe at 8, 12 and 16
# host threads, twice (no split runs).  Each GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-adgather}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_adapter.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_adapter.log 2>&1 &&
timeout -k 10 500 python -u tools/wall_probe.py --out $OUT --workloads c3,c5 --threads 8,12,16,8,12,16 --no-split > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; echo "exit=$rc"; exit $rc
