#!/bin/bash
# r06: k_schur_rows_c variants: descriptors four chunks ahead (OSG_SCHUR_PF=3) and 5 waves per SIMD without
# spills (OSG_SCHUR_WPE=5): bit-identity tests, then the batch bench alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06n}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v -k "variants_bit_identical and (PF or WPE)" --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf2.txt 2>&1 || exit 1
  OSG_SCHUR_PF=3 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf3.txt 2>&1 || exit 1
  OSG_SCHUR_WPE=5 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf2_w5.txt 2>&1 || exit 1
  OSG_SCHUR_PF=3 OSG_SCHUR_WPE=5 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf3_w5.txt 2>&1 || exit 1
done
echo "exit=0"
