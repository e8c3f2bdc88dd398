#!/bin/bash
# LBA batch throughput with the per-kernel split, default and per-column factorisation (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03lbaq}
mkdir -p $OUT
cd $R
TS=1,4 BS=64 KT=1 timeout -k 10 300 python3 tools/lba_batch_bench.py > $OUT/lba_default.txt 2>&1 &&
OSG_LBA_CHOL=0 TS=1,4 BS=64 KT=1 timeout -k 10 300 python3 tools/lba_batch_bench.py > $OUT/lba_percol.txt 2>&1
echo "exit=$?"
