#!/bin/bash
# k_chol_dense variants: 16 waves with a 2-step operand ring (default) and 8 waves with a 3-step ring
# (OSG_CHOL_DENSE_NT=512), against the column launches (OSG_CHOL_DENSE=0): the BA GPU tests under both
# variants, then 64 C4 windows at 1 and 8 host threads with per-kernel HIP-event times, alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-choldense2}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_ba.log 2>&1 || { echo "pytest failed"; exit 1; }
OSG_CHOL_DENSE_NT=512 timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lba or chol" > $OUT/pytest_ba_512.log 2>&1 || { echo "pytest 512 failed"; exit 1; }
run() { local name=$1; shift; env "$@" TS=1,8 BS=64 KT=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/lba_$name.txt 2>&1; }
run d1024 && run d512 OSG_CHOL_DENSE_NT=512 && run column OSG_CHOL_DENSE=0 && run d1024b && run d512b OSG_CHOL_DENSE_NT=512
rc=$?; echo "exit=$rc"; exit $rc
