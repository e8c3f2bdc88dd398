#!/bin/bash
# C2 frame-batched kernel sweep: LDS-broadcast vs scalar-load rows (OSG_TOP2_BATCH_SCALAR) x queries
# per lane (OSG_TOP2_BATCH_QL) x frames per launch.
set -o pipefail
OUT=${1:-gpurun_out/c2sweep}
mkdir -p $OUT
for sc in 0 1; do
for ql in 1 2 4; do
  for b in 64 256; do
    OSG_TOP2_BATCH_SCALAR=$sc OSG_TOP2_BATCH_QL=$ql timeout -k 10 120 python bench.py --no-cpu --no-frames --no-ba \
      --no-gba --no-stream --steps 50 --warmup 5 --c2-batch $b > $OUT/sc${sc}_ql${ql}_b${b}.json 2> $OUT/sc${sc}_ql${ql}_b${b}.err || exit $?
  done
done
done
