#!/bin/bash
# Stereo: the GPU parity tests, then the adapter wall probe (1 and 16 host threads, host phases at 1).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-stereo}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stereo.py tests/test_stereo_fisheye.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_stereo.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -u tools/wall_probe.py --out $OUT --workloads stereo --threads 1,16 > $OUT/stereo_probe.jsonl 2> $OUT/stereo_probe.err
rc=$?; rm -f $OUT/*.arrays; echo "exit=$rc"; exit $rc
