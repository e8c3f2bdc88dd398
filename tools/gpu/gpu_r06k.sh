#!/bin/bash
# r06: k_schur_rows_c with its gathers two groups ahead (OSG_SCHUR_PF=2) against one group ahead: the variant's
# bit-identity test, then the batch bench alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06k}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "variants_bit_identical and PF" --timeout 170 --timeout-method thread > $OUT/pytest_pf.log 2>&1 || exit 1
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf1.txt 2>&1 || exit 1
  OSG_SCHUR_PF=2 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf2.txt 2>&1 || exit 1
done
echo "exit=0"
