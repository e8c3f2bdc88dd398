#!/bin/bash
# The adapter's single-walk grid CSR and deeper MapPoint prefetch: the adapter GPU tests, then the C3 / C5
# wall probe at 16 host threads, twice.  Each GPU step has its own time limit; the chain stops at the first
# failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-adc5}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_adapter.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/wall_probe.py --out $OUT --workloads c5,c3 --threads 16,16 --no-split > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; rm -f $OUT/*.arrays; echo "exit=$rc"; exit $rc
