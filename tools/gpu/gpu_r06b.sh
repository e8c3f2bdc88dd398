#!/bin/bash
# r06: compact-factor Schur A/B (LBA GPU tests, then the C4 batch bench compact / whole-Hpl / compact)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06b}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "lba" --timeout 170 --timeout-method thread > $OUT/pytest_lba.log 2>&1 &&
KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_compact.txt 2>&1 &&
OSG_LBA_HPL=1 KT=1 TS=1 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_full.txt 2>&1 &&
KT=1 TS=1,8 BS=64 REPS=3 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/lba_compact2.txt 2>&1
echo "exit=$?"
