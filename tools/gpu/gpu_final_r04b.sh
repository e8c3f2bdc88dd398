#!/bin/bash
# Late-r04 check (one gpurun call, prebuilt library): the BA GPU tests, the LBA PMC passes
# (tools/gpu/gpu_lba_pmc.sh -> lba_pmc.json), the default bench line reading that file, and the same
# bench under rocprofv3 --kernel-trace --stats.  Each GPU step has its own time limit and the chain
# stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04b}
mkdir -p $OUT
echo pytest > $OUT/progress &&
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_ba.log 2>&1 &&
echo pmc > $OUT/progress &&
bash $R/tools/gpu/gpu_lba_pmc.sh $(basename $OUT)/pmc > $OUT/pmc.log 2>&1 &&
echo bench > $OUT/progress &&
timeout -k 10 400 python bench.py --schur-pmc $OUT/pmc/lba_pmc.json > $OUT/bench.json 2> $OUT/bench.err &&
echo trace > $OUT/progress &&
cd /tmp && timeout -k 10 450 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --no-wall --schur-pmc $OUT/pmc/lba_pmc.json > $OUT/bench_under_trace.json 2> $OUT/trace.err
rc=$?; echo "exit=$rc"; exit $rc
