#!/bin/bash
# r06: k_schur_rows_c's staging loading its blocks from padded per-segment slots (issued with rs_info, not after it)
# against the previous tree's library (build/ab/pre6), alternating; the BA GPU tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06s2}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2 3; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_new.txt 2>&1 || exit 1
  OSG_LIB_PATH=$PWD/build/ab/pre6/liborbslam3_amd.so KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pre.txt 2>&1 || exit 1
done
echo "exit=0"
