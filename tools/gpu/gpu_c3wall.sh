#!/bin/bash
# C3 adapter wall probe: 1 and 16 host threads, gathers timed alone, the library's host phases at 1 thread.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-c3wall}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/wall_probe.py --out $OUT --workloads c3 --threads 1,16 > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; rm -f $OUT/*.arrays; echo "exit=$rc"; exit $rc
