#!/bin/bash
# Kernel trace + stats of the default bench without the C++ adapter wall runs (their child processes
# would run under the profiler too).  A heartbeat file shows the run is alive during long stages.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03trace}
mkdir -p $OUT
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
cd /tmp &&
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --no-wall > $OUT/bench_under_trace.json 2> $OUT/trace.err
rc=$?
kill $HB
echo "exit=$rc"
exit $rc
