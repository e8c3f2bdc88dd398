#!/bin/bash
# End of r06, final tree: the whole GPU suite and smoke, then the driver's bench command and the same bench
# under rocprofv3 --kernel-trace --stats.  Each GPU step has its own time limit; the chain stops at the first
# failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06final}
mkdir -p $OUT
cd $R
echo suite > $OUT/progress &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo bench > $OUT/progress &&
timeout -k 10 450 python bench.py --gpus 1 --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err &&
echo trace > $OUT/progress &&
cd /tmp && timeout -k 10 450 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --no-wall --detail $OUT/trace_detail.json > $OUT/bench_under_trace.json 2> $OUT/trace.err
rc=$?; gzip -f $OUT/trace/trace_kernel_trace.csv 2>/dev/null; echo "exit=$rc"; exit $rc
