#!/bin/bash
# The BA GPU tests (LBA / GBA parity, variants, pose) and the golden BA fixtures on the current build.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-batests}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "exit=$rc"; exit $rc
