#!/bin/bash
# BA parity tests, the LBA batch timing and the FP64 latency microbenchmark (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03ba}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_ba_gpu.py $R/tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 &&
TS=3 BS=64 timeout -k 10 200 python3 $R/tools/lba_batch_bench.py > $OUT/lba.jsonl 2> $OUT/lba.err &&
hipcc --offload-arch=gfx950 -O3 $R/tools/micro/f64_latency.hip -o /tmp/f64lat && timeout -k 10 60 /tmp/f64lat > $OUT/f64_latency.txt 2>&1
echo "exit=$?"
