#!/bin/bash
# FP4 top-2 with the delayed key-pair schedule (OSG_TOP2_MFMA_SHAPE=6) against the default, the top-2 and
# BA GPU tests.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05h}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_top2_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_top2.log 2>&1 || { echo "top2 tests failed"; exit 1; }
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for sh in 0 6 0 6; do
  OSG_TOP2_MFMA_SHAPE=$sh timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_$sh.json >> $OUT/c2_$sh.jsonl 2>> $OUT/bench.err || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_ba.log 2>&1
rc=$?; echo "exit=$rc"; exit $rc
