#!/bin/bash
# r06: XCD-aware graph placement (OSG_LBA_XCD=1) against the default grid on the compact factor (the partner
# M' gathers of a 50-KF window are 2.4 MB, one XCD's L2 is 4 MB), alternating, with gathers 1 / 2 groups ahead
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06l}; mkdir -p $OUT
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_def.txt 2>&1 || exit 1
  OSG_LBA_XCD=1 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_xcd.txt 2>&1 || exit 1
  OSG_LBA_XCD=1 OSG_SCHUR_PF=2 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_xcd_pf2.txt 2>&1 || exit 1
done
KT=1 TS=8 BS=64 REPS=6 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_def_t8.txt 2>&1 || exit 1
OSG_LBA_XCD=1 KT=1 TS=8 BS=64 REPS=6 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_xcd_t8.txt 2>&1 || exit 1
echo "exit=0"
