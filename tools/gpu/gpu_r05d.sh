#!/bin/bash
# r05: ORB GPU tests (the reference's bit_pattern_31_ table, FAST slot bound), smoke, the adapter wall
# probe (16 threads, 64/128/256 frames per call), then the driver's bench command.  Each GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05d}
mkdir -p $OUT
cd $R
echo orb > $OUT/progress &&
timeout -k 10 400 python -u -m pytest tests/test_orb.py tests/test_orb_batch.py tests/test_orb_detect.py tests/test_orb_pyramid.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_orb.log 2>&1 &&
echo smoke > $OUT/progress &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo wall > $OUT/progress &&
timeout -k 10 400 python -u tools/wall_probe.py --out $OUT/wall --threads 16 --frames 64,128,256 --no-split > $OUT/wall_probe.jsonl 2> $OUT/wall_probe.err &&
echo bench > $OUT/progress &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "exit=$rc"; exit $rc
