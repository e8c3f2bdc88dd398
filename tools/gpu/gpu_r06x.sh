#!/bin/bash
# r06: k_linearize's identity shortcut for landmark-ordered edges (default) against the lm_e lookup
# (OSG_LBA_LMIDENT=0), and k_schur_rows_c with descriptors four chunks ahead (OSG_SCHUR_PF=3) re-measured
# now that every form is spill-free; variant bit-identity tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06x}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "variants_bit_identical and (LMIDENT or PF)" --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_def.txt 2>&1 || exit 1
  OSG_LBA_LMIDENT=0 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_lme.txt 2>&1 || exit 1
  OSG_SCHUR_PF=3 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf3.txt 2>&1 || exit 1
  OSG_SCHUR_PF=4 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $OUT/lba_pf4.txt 2>&1 || exit 1
done
echo "exit=0"
