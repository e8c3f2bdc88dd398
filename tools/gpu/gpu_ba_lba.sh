#!/bin/bash
# BA parity tests, then the LBA batch throughput with its per-kernel split (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03balba}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 &&
TS=1,4 BS=64 KT=1 timeout -k 10 300 python3 tools/lba_batch_bench.py > $OUT/lba_default.txt 2>&1
echo "exit=$?"
