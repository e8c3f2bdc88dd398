#!/bin/bash
# r06: k_schur_rows_c with its wave's descriptors preloaded one per lane and branch-free loads
# (OSG_SCHUR_PF=4) against the default (PF 2): the bit-identity test, then alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06y}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "variants_bit_identical and PF" --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2 3; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_def.txt 2>&1 || exit 1
  OSG_SCHUR_PF=4 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf4.txt 2>&1 || exit 1
done
echo "exit=0"
