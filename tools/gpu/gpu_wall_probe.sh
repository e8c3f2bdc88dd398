#!/bin/bash
# Adapter wall-rate probe (tools/wall_probe.py): C3 / C5 at 1, 8, 16 host threads with the gathers
# timed alone and the library's host phases.  One GPU step with its own time limit.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-wallp}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u tools/wall_probe.py --out $OUT ${2:+--threads $2} > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; echo "exit=$rc"; exit $rc
