#!/bin/bash
# FP4 block-scaled top-2: the operand-map probe, the FP4 vs I8 MFMA chain rate, the top-2 GPU tests
# (I8 and FP4 variants), then the headline step with OSG_TOP2_FP4=0 / 1.  Each GPU step has its own time
# limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-fp4}
mkdir -p $OUT
cd $R
[ -n "$LAYOUT" ] && { timeout -k 10 60 tools/micro/mfma_fp4_layout > $OUT/layout.txt 2>&1 || exit 1; }
timeout -k 10 120 tools/micro/mfma_fp4_rate > $OUT/rate.jsonl 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_top2_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_top2.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_top2.log
ARGS="--no-frames --no-ba --no-gba --no-cpu --no-stream --steps 200 --warmup 20"
for v in 0 1 0 1; do
  OSG_TOP2_FP4=$v timeout -k 10 200 python bench.py $ARGS --detail $OUT/c2_fp4_$v.json >> $OUT/c2_fp4_$v.jsonl 2>> $OUT/bench.err || exit 1
done
echo "exit=0"
