#!/bin/bash
# Diagonal-tile elimination four columns per barrier (OSG_CHOL_ELIM=4) against two (default): the BA GPU tests
# under ELIM=4, single-window phase timestamps, 64-window LBA at 8 host threads, and the global BA stages.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-elim4}
mkdir -p $OUT
cd $R
OSG_CHOL_ELIM=4 timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_ba_elim4.log 2>&1 || { echo "pytest failed"; exit 1; }
OSG_CHOL_ELIM=4 OSG_LBA_PROFILE=2 TS=1 BS=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/phase_dense4.txt 2>&1 &&
OSG_CHOL_ELIM=4 OSG_CHOL_DENSE=0 OSG_LBA_PROFILE=2 TS=1 BS=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/phase_col4.txt 2>&1 || exit 1
run() { local name=$1; shift; env "$@" TS=1,8 BS=64 KT=1 timeout -k 10 240 python tools/lba_batch_bench.py > $OUT/lba_$name.txt 2>&1; }
run e2 && run e4 OSG_CHOL_ELIM=4 && run e2b && run e4b OSG_CHOL_ELIM=4 || exit 1
gba() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py --only global_ba,global_ba_map,global_ba_loop --no-cpu --steps 20 --warmup 5 --detail $OUT/gba_$name.json > $OUT/gba_$name.jsonl 2>> $OUT/gba.err; }
gba e2 && gba e4 OSG_CHOL_ELIM=4
rc=$?; echo "exit=$rc"; exit $rc
