#!/bin/bash
# r06: against the previous tree's library (build/ab/pre3 through OSG_LIB_PATH), alternating:
#   the FP4 top-2 epilogue with key_push2f (v_med3_f32 + v_min3_i32: 22 VALU ops per tile instead of 30),
#   k_update_c / k_update with Dinv in registers (no scratch);
# the top-2 / shard / BA GPU tests first (bit-exact top-2, BA parity)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06t}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_top2_gpu.py tests/test_shard_dist.py tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_new.json >> $OUT/c2_new.jsonl 2>> $OUT/bench.err || exit 1
  OSG_LIB_PATH=$PWD/build/ab/pre3/liborbslam3_amd.so timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_pre.json >> $OUT/c2_pre.jsonl 2>> $OUT/bench.err || exit 1
done
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_new.txt 2>&1 || exit 1
  OSG_LIB_PATH=$PWD/build/ab/pre3/liborbslam3_amd.so KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pre.txt 2>&1 || exit 1
done
echo "exit=0"
