#!/bin/bash
# k_pose_opt phase counters (profiling build build/pprof) alternating OSG_POSE_LANES; time-limited.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06pp}
mkdir -p $OUT
cd $R
OSG_LIB_PATH=$R/build/pprof/liborbslam3_amd.so timeout -k 10 200 python3 -u tools/pose_phase_ab.py OSG_POSE_LANES > $OUT/pose_phase.jsonl 2> $OUT/pose_phase.err || { echo "phase probe failed"; tail $OUT/pose_phase.err; exit 1; }
cat $OUT/pose_phase.jsonl
