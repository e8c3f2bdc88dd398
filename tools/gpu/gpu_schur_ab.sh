#!/bin/bash
# k_schur_rows A/B (one gpurun call): 64 C4 windows, per-kernel device times of one batch and the
# 1- / 8-thread LM iteration rates, MFMA form then the VALU form (OSG_SCHUR_VALU=1); then the LBA
# GPU parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-schur_ab}
mkdir -p $O
for v in 0 1; do
  echo "# OSG_SCHUR_VALU=$v" >> $O/ab.txt
  OSG_SCHUR_VALU=$v KT=1 TS=1,8 BS=64 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $O/ab.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_ba.log 2>&1
echo "exit=$?"
