#!/bin/bash
# One GPU call: build, parity tests, smoke, bench, rocprof kernel trace.  Each GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-run}
mkdir -p $OUT
make -j16 > $OUT/build.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu ${BENCH_ARGS} > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
echo "exit=$?"
