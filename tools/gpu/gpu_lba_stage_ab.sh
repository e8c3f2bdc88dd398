#!/bin/bash
# LBA Schur A/B on one GPU box (64 C4 windows, one host thread, per-kernel HIP-event times):
# k_schur_rows (default), the LDS-staged partner spans (OSG_SCHUR_STAGE=1) alone and with the
# landmark-ordered launch / one window per XCD, then the host phase split at 1 and 8 host threads.
set -o pipefail
OUT=gpurun_out/${1:-lba_ab}
mkdir -p $OUT
run() { local name=$1; shift; env "$@" TS=1 BS=64 KT=1 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/$name.txt 2>&1; }
run base &&
run stage OSG_SCHUR_STAGE=1 &&
run stage_order OSG_SCHUR_STAGE=1 OSG_SCHUR_ORDER=1 &&
run stage_order_xcd OSG_SCHUR_STAGE=1 OSG_SCHUR_ORDER=1 OSG_LBA_XCD=1 &&
OSG_LBA_PROFILE=1 TS=1,8 BS=64 timeout -k 10 200 python tools/lba_batch_bench.py > $OUT/prof.txt 2>&1
echo "exit=$?"
