#!/bin/bash
# r06: FP4 top-2 workgroup shapes with the key_push2f epilogue: the default {16,1,256,3} against PIPE 0
# (shape 2), {8,1,256,3} (shape 9, two workgroups per CU) and {8,1,256,1} (shape 4), alternating; the new
# shape's bit-exactness tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06u}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_top2_gpu.py -m gpu -x -q -k "SHAPE=9" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for rep in 1 2; do
  for sh in 0 2 9 4; do
    OSG_TOP2_MFMA_SHAPE=$sh timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_$sh.json >> $OUT/c2_$sh.jsonl 2>> $OUT/bench.err || exit 1
  done
done
echo "exit=0"
