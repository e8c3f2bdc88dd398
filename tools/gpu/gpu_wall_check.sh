#!/bin/bash
# Adapter GPU tests (incl. ComputeBoW and the batched entries), then the frame workloads of bench.py
# with the C++ adapter wall rate, at two host-thread counts (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03wall}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_adapter.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-stream --no-ba --no-gba --frame-reps 2 --cpu-seconds 4 --wall-threads 8 > $OUT/bench_t8.json 2> $OUT/bench_t8.err &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-stream --no-ba --no-gba --no-cpu --frame-reps 2 --wall-threads 16 --wall-frames 128 > $OUT/bench_t16.json 2> $OUT/bench_t16.err
echo "exit=$?"
