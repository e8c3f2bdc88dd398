#!/bin/bash
# SearchByBoW query rows gathered straight into the pinned block: the matcher and adapter GPU tests, then
# the C3 wall probe at 1 and 16 host threads (the 1-thread split run carries the library's host phases).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-bowrows}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_match_gpu.py tests/test_adapter.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/wall_probe.py --out $OUT --workloads c3 --threads 1,16,16 > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; rm -f $OUT/*.arrays; echo "exit=$rc"; exit $rc
