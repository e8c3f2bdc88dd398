#!/bin/bash
# r06: the FP4 top-2 kernel time against the train rows per frame (1000 / 2000 / 4000, 2000 queries, 1024 frames):
# the intercept is the per-workgroup fixed cost (LUT, query fragments, first chunk, output)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06z}; mkdir -p $OUT
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 100 --warmup 10"
for rep in 1 2; do
  for nt in 1000 2000 4000; do
    timeout -k 10 200 python bench.py $ARGS --nt $nt --detail $OUT/c2_$nt.json >> $OUT/c2_$nt.jsonl 2>> $OUT/bench.err || exit 1
  done
done
echo "exit=0"
