#!/bin/bash
# r06: the persistent FP4 top-2 (OSG_TOP2_MFMA_SHAPE=13: one workgroup per CU over the items, the next item's
# first chunk and (r06p3) its query rows by LDS-DMA loaded during the last one) against the default: its bit-exactness tests, then alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06p3}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_top2_gpu.py -m gpu -x -q -k "MFMA_SHAPE and 13" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for rep in 1 2 3; do
  for sh in 0 13; do
    OSG_TOP2_MFMA_SHAPE=$sh timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_$sh.json >> $OUT/c2_$sh.jsonl 2>> $OUT/bench.err || exit 1
  done
done
echo "exit=0"
