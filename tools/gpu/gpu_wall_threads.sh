#!/bin/bash
# C3 / C5 adapter wall rate against the host-thread count (the bench uses one thread per CPU the job may
# use, 16 on the box): 8, 12, 16, alternating twice, no split runs.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-wallthr}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/wall_probe.py --out $OUT --workloads c3,c5 --threads 8,12,16,8,12,16 --no-split > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; echo "exit=$rc"; exit $rc
