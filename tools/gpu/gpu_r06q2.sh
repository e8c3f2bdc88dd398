#!/bin/bash
# r06: the FP4 top-2 default (PIPE 3) with the pipelined block also over a partial chunk's full tiles (a
# compile-time tile count per case) against the previous tree's library (build/ab/pre5): every top-2 GPU test,
# then alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06q2}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_top2_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_new.json >> $OUT/c2_new.jsonl 2>> $OUT/bench.err || exit 1
  OSG_LIB_PATH=$PWD/build/ab/pre5/liborbslam3_amd.so timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_pre.json >> $OUT/c2_pre.jsonl 2>> $OUT/bench.err || exit 1
done
echo "exit=0"
