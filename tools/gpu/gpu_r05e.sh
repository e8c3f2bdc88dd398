#!/bin/bash
# Late r05, FP4 default: the top-2 GPU tests, the FP4 workgroup shapes A/B on the headline step, the FP4
# kernel's FETCH_SIZE / WRITE_SIZE passes (-> pmc_traffic_fp4.json), then the stereo adapter wall probe
# with the library's host phases.  Every GPU step has its own time limit; the chain stops at the first
# failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05e}
mkdir -p $OUT
cd $R
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream"
timeout -k 10 300 python -u -m pytest tests/test_top2_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_top2.log 2>&1 || { echo "pytest failed"; exit 1; }
for sh in 0 1 2 4 5 0; do
  OSG_TOP2_MFMA_SHAPE=$sh timeout -k 10 200 python bench.py $ARGS --steps 200 --warmup 20 --detail $OUT/shape_$sh.json >> $OUT/shape_$sh.jsonl 2>> $OUT/bench.err || exit 1
done
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS --steps 20 --warmup 5 > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS --steps 20 --warmup 5 > $OUT/write.log 2>&1 || exit 1
python3 $R/tools/pmc_traffic.py $(find $OUT/fetch -name '*counter_collection.csv' | head -1) $(find $OUT/write -name '*counter_collection.csv' | head -1) $OUT/pmc_traffic_fp4.json || exit 1
rm -rf $OUT/fetch $OUT/write
cd $R
timeout -k 10 300 python -u tools/wall_probe.py --out $OUT --workloads stereo --threads 1,16 > $OUT/stereo_probe.jsonl 2> $OUT/stereo_probe.err
rc=$?; echo "exit=$rc"; exit $rc
