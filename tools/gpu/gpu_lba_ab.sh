#!/bin/bash
# LBA Schur A/B on one box: BA parity tests, then the batch bench with the FP64-MFMA Schur product
# (default) and the VALU one (OSG_SCHUR_VALU=1), per-kernel HIP-event times of one batch (KT=1).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lba_ab}; mkdir -p $OUT
make -j16 > $OUT/build.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_c1_mono_chain.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ba.log 2>&1 &&
KT=1 TS=1,4 BS=64 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_mfma.txt 2>&1 &&
OSG_SCHUR_VALU=1 KT=1 TS=1,4 BS=64 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_valu.txt 2>&1
echo "exit=$?"
