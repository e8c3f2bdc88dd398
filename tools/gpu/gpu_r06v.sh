#!/bin/bash
# r06: FP4 top-2 chunk shapes with the key_push2f epilogue: the default {16,1,256,3} against 512-row chunks
# (shape 10) and the pipelined block also over a partial chunk's full tiles (PIPE 5: shapes 11, 12), alternating;
# shape's bit-exactness tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06v}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_top2_gpu.py -m gpu -x -q -k "MFMA_SHAPE" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for rep in 1 2; do
  for sh in 0 10 11 12; do
    OSG_TOP2_MFMA_SHAPE=$sh timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_$sh.json >> $OUT/c2_$sh.jsonl 2>> $OUT/bench.err || exit 1
  done
done
echo "exit=0"
