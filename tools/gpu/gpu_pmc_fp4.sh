#!/bin/bash
# HBM traffic of the default FP4 top-2 kernel: separate FETCH_SIZE and WRITE_SIZE passes over the headline
# step (kernel trace only), reduced by tools/pmc_traffic.py.  Each pass has its own time limit; the chain stops
# at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-pmcfp4}
mkdir -p $OUT
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream"
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS --steps 20 --warmup 5 > $OUT/fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS --steps 20 --warmup 5 > $OUT/write.log 2>&1 &&
python3 $R/tools/pmc_traffic.py $(find $OUT/fetch -name '*counter_collection.csv' | head -1) $(find $OUT/write -name '*counter_collection.csv' | head -1) $OUT/pmc_traffic_fp4.json
rc=$?; rm -rf $OUT/fetch $OUT/write; echo "exit=$rc"; exit $rc
