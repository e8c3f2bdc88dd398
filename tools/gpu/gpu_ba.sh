#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ba}
mkdir -p $OUT
make -j16 > $OUT/build.log 2>&1 &&
timeout -k 10 600 python -m pytest tests/test_ba_gpu.py -x -q > $OUT/pytest_ba.log 2>&1 &&
OSG_LBA_PROFILE=1 timeout -k 10 300 python bench.py --no-cpu --no-stream --steps 50 > $OUT/bench.json 2> $OUT/bench.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-stream --steps 50 --ba-reps 5 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
echo "exit=$?"
