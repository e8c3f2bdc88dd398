#!/bin/bash
# PoseOptimization lane-parallel solve / exp-map update: the pose parity tests (incl. OSG_POSE_LANES=0/1),
# then the single-call / batch A/B alternating OSG_POSE_LANES.  Each GPU step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06pl}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pose" > $OUT/pytest_pose.log 2>&1 || { echo "pose tests failed"; tail -30 $OUT/pytest_pose.log; exit 1; }
tail -3 $OUT/pytest_pose.log
timeout -k 10 300 python3 -u tools/pose_sum_ab.py OSG_POSE_LANES > $OUT/pose_lanes_ab.jsonl 2> $OUT/pose_lanes_ab.err || { echo "pose probe failed"; exit 1; }
cat $OUT/pose_lanes_ab.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['OSG_POSE_LANES'], d['rep'], {k:(v['kernel_us'],v['wall_us'],v['trials']) for k,v in d.items() if k.startswith('single')}, d['batch256_kernel_us'])"
