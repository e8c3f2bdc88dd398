#!/bin/bash
# r06: one 128-byte record per landmark (Hll, b_l, X; the default now) against three arrays (OSG_LBA_LREC=0):
# bit-identity test, the batch bench alternating, and the k_schur_rows_c timeline with the record layout
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06p}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v -k "variants_bit_identical and LREC" --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_rec.txt 2>&1 || exit 1
  OSG_LBA_LREC=0 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_arr.txt 2>&1 || exit 1
done
OSG_LIB_PATH=$PWD/build/srprof/liborbslam3_amd.so OSG_SR_PROF_OUT=$OUT/sr.bin TS=1 BS=64 REPS=1 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/bench_sr.txt 2>&1 &&
python3 tools/sr_prof.py $OUT/sr.bin > $OUT/sr.txt 2>&1 &&
OSG_LBA_LREC=0 OSG_LIB_PATH=$PWD/build/srprof/liborbslam3_amd.so OSG_SR_PROF_OUT=$OUT/sr0.bin TS=1 BS=64 REPS=1 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/bench_sr0.txt 2>&1 &&
python3 tools/sr_prof.py $OUT/sr0.bin > $OUT/sr0.txt 2>&1
rc=$?; echo "exit=$rc"; exit $rc
