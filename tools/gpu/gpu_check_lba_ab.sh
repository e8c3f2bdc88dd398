#!/bin/bash
# One gpurun call: every GPU test, smoke(), then the LBA A/B of tools/gpu/gpu_lba_env_ab.sh (without
# its own test pass) for the variants given as arguments.  Each GPU step has its own time limit and
# the chain stops at the first failure.
#   tools/gpu/gpu_check_lba_ab.sh OUTNAME [VAR=VAL ...]
set -o pipefail
OUT=gpurun_out/${1:-check_ab}
shift
mkdir -p $OUT
echo pytest > $OUT/progress &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo smoke > $OUT/progress &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo ab > $OUT/progress &&
run() { local name=$1; shift; env "$@" TS=1,8 BS=64 KT=1 REPS=${REPS:-4} timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/$name.txt 2>&1; } &&
run base &&
i=0 &&
for v in "$@"; do i=$((i + 1)); run "${i}_${v//[=]/_}" "$v" || exit $?; done
rc=$?; echo "exit=$rc"; exit $rc
