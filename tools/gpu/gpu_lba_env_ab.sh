#!/bin/bash
# LBA A/B on one GPU box: the LBA / GBA GPU tests, then 64 C4 windows per batch with per-kernel
# HIP-event times (one host thread) and at 8 host threads, for the default build and for each
# environment given as an argument (e.g. OSG_POSE_RED_GATHER=1).
#   tools/gpu/gpu_lba_env_ab.sh OUTNAME [VAR=VAL ...]
set -o pipefail
OUT=gpurun_out/${1:-lba_env_ab}
shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_ba.txt 2>&1 &&
run() { local name=$1; shift; env "$@" TS=1,8 BS=64 KT=1 REPS=${REPS:-4} timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/$name.txt 2>&1; }
run base &&
i=0
for v in "$@"; do i=$((i + 1)); run "${i}_${v//[=]/_}" "$v" || exit $?; done &&
run base2
rc=$?; echo "exit=$rc"; exit $rc
