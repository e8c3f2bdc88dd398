#!/bin/bash
# Round-end check (one gpurun call, prebuilt library): every GPU test, smoke(), the default bench
# line, and the same bench under rocprofv3 --kernel-trace --stats (profiles/r04_kernel_stats.csv).
# Each GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04final}
mkdir -p $OUT
echo pytest > $OUT/progress &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo smoke > $OUT/progress &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo bench > $OUT/progress &&
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
echo trace > $OUT/progress &&
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py > $OUT/bench_under_trace.json 2> $OUT/trace.err
echo "exit=$?"
