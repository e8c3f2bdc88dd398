#!/bin/bash
# LocalBA windows per batch x host threads (tools/lba_batch_bench.py, C4 windows), alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-lbabs}
mkdir -p $OUT
cd $R
run() { TS=$1 BS=$2 timeout -k 10 240 python tools/lba_batch_bench.py >> $OUT/t$1_b$2.txt 2>&1; }
run 8 64 && run 8 128 && run 8 192 && run 8 256 && run 16 64 && run 16 128 && run 8 64 && run 8 128 && run 8 256
rc=$?; echo "exit=$rc"; exit $rc
