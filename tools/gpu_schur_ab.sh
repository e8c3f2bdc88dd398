#!/bin/bash
# k_schur_rows A/B: the FP64 MFMA form against OSG_SCHUR_VALU=1 on the 64-window C4 batch (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03schurab}
mkdir -p $OUT
cd $R
for v in 0 1 0 1; do
  OSG_SCHUR_VALU=$v TS=1 BS=64 KT=1 timeout -k 10 200 python3 tools/lba_batch_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/VALU=$v: /" >> $OUT/ab.txt || exit 1
done
echo "exit=$?"
