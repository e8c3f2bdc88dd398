#!/bin/bash
# Fused dense Cholesky (k_chol_dense) against the per-column launches (OSG_CHOL_DENSE=0): the BA GPU
# tests, then 64 C4 windows at 1 and 8 host threads with per-kernel HIP-event times, alternating.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-choldense}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_ba.log 2>&1 || { echo "pytest failed"; exit 1; }
run() { local name=$1; shift; env "$@" TS=1,8 BS=64 KT=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/$name.txt 2>&1; }
run dense &&
run column OSG_CHOL_DENSE=0 &&
run dense2 &&
run column2 OSG_CHOL_DENSE=0
rc=$?; echo "exit=$rc"; exit $rc
