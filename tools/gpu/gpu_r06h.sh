#!/bin/bash
# r06: same-box A/B of the LBA Schur forms: the current compact kernel (v5), the whole-Hpl form (OSG_LBA_HPL=1)
# and the first compact form (build/ab/v1, camera-frame M, loaded through OSG_LIB_PATH), alternating; LBA tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06h}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "lba or gba" --timeout 170 --timeout-method thread > $OUT/pytest_lba.log 2>&1 || exit 1
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_v5.txt 2>&1 || exit 1
  OSG_LBA_HPL=1 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_full.txt 2>&1 || exit 1
  OSG_LIB_PATH=$PWD/build/ab/v1/liborbslam3_amd.so KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_v1.txt 2>&1 || exit 1
done
echo "exit=0"
