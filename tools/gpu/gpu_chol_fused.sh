#!/bin/bash
# One-workgroup factorisations (k_chol_dense, k_chol_env) against the per-column launches
# (OSG_CHOL_DENSE=0): the BA GPU tests, then 64 C4 windows at 1 and 8 host threads with per-kernel
# HIP-event times, then the global BA stages of bench.py, alternating.  Every GPU step has its own time
# limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-cholfused}
mkdir -p $OUT
cd $R
timeout -k 10 120 tools/micro/mfma_fp4_rate > $OUT/fp4_rate.jsonl 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_ba.log 2>&1 || { echo "pytest failed"; exit 1; }
run() { local name=$1; shift; env "$@" TS=1,8 BS=64 KT=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/lba_$name.txt 2>&1; }
gba() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --only global_ba,global_ba_map,global_ba_loop --no-cpu --steps 20 --warmup 5 --detail $OUT/gba_$name.json > $OUT/gba_$name.jsonl 2>> $OUT/gba.err; }
run fused && run column OSG_CHOL_DENSE=0 && run fused2 && run column2 OSG_CHOL_DENSE=0 &&
gba fused && gba column OSG_CHOL_DENSE=0
rc=$?; echo "exit=$rc"; exit $rc
