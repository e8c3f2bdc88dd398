#!/bin/bash
# r06: the FP4 top-2 epilogue with key_push2f (v_med3_f32 + v_min3_i32: 22 VALU ops per tile instead of 30)
# against the previous tree's library (build/ab/pre3), alternating; then every top-2 GPU test (bit-exact)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06s}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_top2_gpu.py tests/test_shard_dist.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_new.json >> $OUT/c2_new.jsonl 2>> $OUT/bench.err || exit 1
  OSG_LIB_PATH=$PWD/build/ab/pre3/liborbslam3_amd.so timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_pre.json >> $OUT/c2_pre.jsonl 2>> $OUT/bench.err || exit 1
done
echo "exit=0"
