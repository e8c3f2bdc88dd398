#!/bin/bash
# End of r05: the pose tests and the pose A/B + phase probes of the barrier-trimmed passes, then the whole
# GPU suite in one process and smoke.  Each GPU step has its own time limit; the chain stops at the first
# failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05n}
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pose" > $OUT/pytest_pose.log 2>&1 &&
timeout -k 10 200 python3 -u tools/pose_sum_ab.py > $OUT/pose_ab.jsonl 2> $OUT/pose_ab.err &&
OSG_PROBE_LIB=$R/build/prof/liborbslam3_amd.so timeout -k 10 150 python3 -u tools/latency_probe.py > $OUT/pose_prof.jsonl 2> $OUT/pose_prof.err &&
timeout -k 10 850 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "exit=$rc"; exit $rc
