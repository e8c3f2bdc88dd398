#!/bin/bash
# XCD-aware LBA graph placement A/B: BA parity tests, then the batch bench with OSG_LBA_XCD=1 (default)
# and 0, per-kernel HIP-event times of one 64-window batch; each GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lba_xcd}; mkdir -p $OUT
make -j16 > $OUT/build.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py tests/test_c1_mono_chain.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ba.log 2>&1 &&
KT=1 TS=1,4 BS=64 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_xcd1.txt 2>&1 &&
OSG_LBA_XCD=0 KT=1 TS=1,4 BS=64 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_xcd0.txt 2>&1
echo "exit=$?"
