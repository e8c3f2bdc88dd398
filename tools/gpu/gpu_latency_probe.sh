#!/bin/bash
# Single-call latency probes (tools/latency_probe.py, with OSG_MATCH_PROFILE=1) and the batched LBA
# host/device split (OSG_LBA_PROFILE=1).  Each GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-probe}; mkdir -p $OUT
make -j16 > $OUT/build.log 2>&1 &&
OSG_MATCH_PROFILE=1 timeout -k 10 120 python -u tools/latency_probe.py > $OUT/latency.jsonl 2> $OUT/latency.err &&
OSG_LBA_PROFILE=1 BS=1,64 timeout -k 10 180 python -u tools/lba_batch_bench.py > $OUT/lba_batch.txt 2>&1
echo "exit=$?"
