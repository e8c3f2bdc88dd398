#!/bin/bash
# r05: BA GPU tests (k_init_state, ctl through the copy kernel), the adapter wall probe (1 and 16
# host threads, library host phases), then the driver's bench command.  Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05c}
mkdir -p $OUT
cd $R
echo ba > $OUT/progress &&
timeout -k 10 500 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ba.log 2>&1 &&
echo wall > $OUT/progress &&
timeout -k 10 400 python -u tools/wall_probe.py --out $OUT/wall --threads 1,16 > $OUT/wall_probe.jsonl 2> $OUT/wall_probe.err &&
echo bench > $OUT/progress &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "exit=$rc"; exit $rc
