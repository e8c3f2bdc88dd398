#!/bin/bash
# r06: the landmark record layout (OSG_LBA_LREC, default on), the spill-free staging order and the hoisted first
# gathers (OSG_SCHUR_HOIST=1): bit-identity tests, then the batch bench alternating against the previous tree's
# library (build/ab/pre through OSG_LIB_PATH), then the k_schur_rows_c timeline of the new default
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06q}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v -k "(variants_bit_identical and (LREC or HOIST or PF)) or compact_factor or two_camera_rig" --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_new.txt 2>&1 || exit 1
  OSG_LIB_PATH=$PWD/build/ab/pre/liborbslam3_amd.so KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pre.txt 2>&1 || exit 1
  OSG_LBA_LREC=0 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_arr.txt 2>&1 || exit 1
  OSG_SCHUR_HOIST=1 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_hoist.txt 2>&1 || exit 1
done
OSG_LIB_PATH=$PWD/build/srprof/liborbslam3_amd.so OSG_SR_PROF_OUT=$OUT/sr.bin TS=1 BS=64 REPS=1 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/bench_sr.txt 2>&1 &&
python3 tools/sr_prof.py $OUT/sr.bin > $OUT/sr.txt 2>&1
rc=$?; echo "exit=$rc"; exit $rc
