#!/bin/bash
# One-frame-per-call ORB stages at 4, 8 and 16 host threads (bench.py --ba-threads).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-orbthr}
mkdir -p $OUT
cd $R
for t in 4 8 16 4; do
  timeout -k 10 300 python bench.py --only frames_orb,frames_orb_detect --no-cpu --steps 20 --warmup 5 --ba-threads $t --detail $OUT/orb_t$t.json >> $OUT/orb_t$t.jsonl 2>> $OUT/orb.err || exit 1
done
echo "exit=0"
