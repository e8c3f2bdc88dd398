#!/bin/bash
# r06: the compact per-block factor.  BA GPU tests, then the C4 batch bench (per-kernel HIP-event split)
# with the compact factor (default) and the whole-Hpl form (OSG_LBA_HPL=1), alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06a}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest_ba.log 2>&1 &&
KT=1 TS=1,8 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_compact.txt 2>&1 &&
OSG_LBA_HPL=1 KT=1 TS=1,8 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_full.txt 2>&1 &&
KT=1 TS=1,8 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_compact2.txt 2>&1
echo "exit=$?"
