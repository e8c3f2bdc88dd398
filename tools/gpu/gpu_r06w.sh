#!/bin/bash
# r06: memory round trips cut in k_schur_pairs (rotation operands loaded before the sums, four partials per
# round trip), k_pose_red (the next edge record one edge ahead) and k_update_c (the next piece's block one
# piece ahead), against the previous tree's library (build/ab/pre4), alternating; the BA GPU tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06w}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_new.txt 2>&1 || exit 1
  OSG_LIB_PATH=$PWD/build/ab/pre4/liborbslam3_amd.so KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pre.txt 2>&1 || exit 1
done
TS=8 BS=64 REPS=6 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_new_t8.txt 2>&1 || exit 1
OSG_LIB_PATH=$PWD/build/ab/pre4/liborbslam3_amd.so TS=8 BS=64 REPS=6 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pre_t8.txt 2>&1 || exit 1
echo "exit=0"
