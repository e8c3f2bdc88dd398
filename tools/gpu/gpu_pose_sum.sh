#!/bin/bash
# PoseOptimization whole-row sums: the pose parity tests (every variant, incl. OSG_POSE_ROWSUM=0/1), the
# A/B probe, then the top-2 tests and the FP4 one-chain A/B (tools/gpu/gpu_fp4_one.sh's steps).  Every GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-posesum}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pose" > $OUT/pytest_pose.log 2>&1 || { echo "pose tests failed"; exit 1; }
timeout -k 10 200 python3 -u tools/pose_sum_ab.py > $OUT/pose_ab.jsonl 2> $OUT/pose_ab.err || { echo "pose probe failed"; exit 1; }
bash tools/gpu/gpu_fp4_one.sh ${1:-posesum}
