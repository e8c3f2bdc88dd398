#!/bin/bash
# PoseOptimization phase counters (library built with `make POSE_PROF=1 OBJDIR=build/objprof
# LIB=build/prof/liborbslam3_amd.so`) through the single-call latency probe.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-poseprof}
mkdir -p $OUT
cd $R
OSG_PROBE_LIB=$R/build/prof/liborbslam3_amd.so timeout -k 10 150 python3 -u tools/latency_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?; echo "exit=$rc"; exit $rc
