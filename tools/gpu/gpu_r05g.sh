#!/bin/bash
# Late r05 final measurement: the driver's bench command (compact stdout line + the full record in
# --detail), then the same bench under rocprofv3 --kernel-trace --stats with the library's SIGSEGV maps
# dump on (OSG_SEGV_MAPS=1).  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05g}
mkdir -p $OUT
cd $R
echo bench > $OUT/progress &&
timeout -k 10 450 python bench.py --gpus 1 --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err &&
echo trace > $OUT/progress &&
export OSG_SEGV_MAPS=1 &&
cd /tmp && timeout -k 10 550 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --no-wall --detail $OUT/trace_detail.json > $OUT/bench_under_trace.json 2> $OUT/trace.err
rc=$?; gzip -f $OUT/trace/trace_kernel_trace.csv 2>/dev/null; echo "exit=$rc"; exit $rc
