#!/bin/bash
# k_schur_rows launch order A/B (one gpurun call): row segments in landmark order (OSG_SCHUR_ORDER=1)
# against pose order, with and without the XCD-aware graph placement (OSG_LBA_XCD=1); 64 C4 windows,
# per-kernel device times of one batch and the 1- / 8-thread LM iteration rates.  Then the LBA GPU
# parity tests with the landmark order.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-schur_order}
mkdir -p $O
for cfg in "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  echo "# OSG_SCHUR_ORDER=$1 OSG_LBA_XCD=$2" >> $O/ab.txt
  OSG_SCHUR_ORDER=$1 OSG_LBA_XCD=$2 KT=1 TS=1,8 BS=64 timeout -k 10 200 python -u tools/lba_batch_bench.py >> $O/ab.txt 2>&1 || exit 1
done
OSG_SCHUR_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_ba.log 2>&1
echo "exit=$?"
