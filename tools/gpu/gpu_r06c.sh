#!/bin/bash
# r06: FP4 top-2 with the wave-uniform skip test (OSG_TOP2_MFMA_SHAPE=8) against the default: the top-2 GPU
# tests, then the headline step alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06c}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_top2_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_top2.log 2>&1 || { echo "top2 tests failed"; exit 1; }
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for sh in 0 8 0 8; do
  OSG_TOP2_MFMA_SHAPE=$sh timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_$sh.json >> $OUT/c2_$sh.jsonl 2>> $OUT/bench.err || exit 1
done
echo "exit=0"
