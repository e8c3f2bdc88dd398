#!/bin/bash
# Profiles for profiles/<tag>_*: (1) kernel-trace + stats of the default bench command,
# (2)/(3) separate --pmc passes for FETCH_SIZE and WRITE_SIZE (counters never combined with traces),
# then per-launch traffic.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
make -j16 > $OUT/build.log 2>&1 &&
cd /tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py > $OUT/bench_under_trace.json 2> $OUT/trace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py --no-cpu --no-ba --steps 20 --warmup 5 > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py --no-cpu --no-ba --steps 20 --warmup 5 > $OUT/write.log 2>&1 &&
python3 $R/tools/pmc_traffic.py $(find $OUT/fetch -name '*counter_collection.csv' | head -1) $(find $OUT/write -name '*counter_collection.csv' | head -1) $OUT/pmc_traffic.json &&
timeout -k 10 300 python3 $R/bench.py --traffic $OUT/pmc_traffic.json > $OUT/bench.json 2> $OUT/bench.err
echo "exit=$?"
