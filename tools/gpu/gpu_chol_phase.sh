#!/bin/bash
# Phase timestamps of the dense factorisation (OSG_LBA_PROFILE=2, one C4 window, first step): k_chol_dense
# (default) and the column launches (OSG_CHOL_DENSE=0); then LocalBA batch size / host threads A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-cholphase}
mkdir -p $OUT
cd $R
OSG_LBA_PROFILE=2 TS=1 BS=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/dense.txt 2>&1 &&
OSG_CHOL_DENSE=0 OSG_LBA_PROFILE=2 TS=1 BS=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/column.txt 2>&1 &&
TS=8 BS=64 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/t8_b64.txt 2>&1 &&
TS=8 BS=128 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/t8_b128.txt 2>&1 &&
TS=4 BS=128 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/t4_b128.txt 2>&1 &&
TS=8 BS=64 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/t8_b64b.txt 2>&1
rc=$?; echo "exit=$rc"; exit $rc
