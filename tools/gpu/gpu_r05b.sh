#!/bin/bash
# r05: the adapter GPU tests (pooled gathers), the global-BA tests (envelope tile store, 9000-KF map),
# then the adapter wall probe at 8 and 16 host threads.  Each GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05b}
mkdir -p $OUT
cd $R
echo adapter > $OUT/progress &&
timeout -k 10 300 python -u -m pytest tests/test_adapter.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_adapter.log 2>&1 &&
echo gba > $OUT/progress &&
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -v -k "gba" --timeout 300 --timeout-method thread > $OUT/pytest_gba.log 2>&1 &&
echo wall > $OUT/progress &&
timeout -k 10 400 python -u tools/wall_probe.py --out $OUT/wall --threads 8,16 > $OUT/wall_probe.jsonl 2> $OUT/wall_probe.err
rc=$?; echo "exit=$rc"; exit $rc
