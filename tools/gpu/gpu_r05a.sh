#!/bin/bash
# r05 first GPU call (prebuilt library): the driver's bench command (compact stdout line + the full
# record in --detail), then the same bench under rocprofv3 --kernel-trace --stats with the library's
# SIGSEGV maps dump on (OSG_SEGV_MAPS=1), so a repeat of r04's k_chol_back launch fault can be mapped
# to its libraries.  Each GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05a}
mkdir -p $OUT
echo bench > $OUT/progress &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err &&
echo trace > $OUT/progress &&
export OSG_SEGV_MAPS=1 &&
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --no-wall --detail $OUT/trace_detail.json > $OUT/bench_under_trace.json 2> $OUT/trace.err
rc=$?; echo "exit=$rc"; exit $rc
