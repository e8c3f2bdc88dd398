#!/bin/bash
# PoseOptimization with the system's LDS reads pinned before the factorisation (a build with -DOSG_POSE_PIN in
# build/pin, loaded through OSG_LIB_PATH) against the default build: the pose tests on the variant, then the
# pose A/B probe alternating the two libraries.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-posepin}
mkdir -p $OUT
cd $R
OSG_LIB_PATH=$R/build/pin/liborbslam3_amd.so timeout -k 10 200 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pose" > $OUT/pytest_pose.log 2>&1 || { echo "pose tests failed"; exit 1; }
for v in base pin base pin; do
  if [ $v = pin ]; then L=$R/build/pin/liborbslam3_amd.so; else L=$R/orb_slam3_comments_ghr_amd/liborbslam3_amd.so; fi
  OSG_LIB_PATH=$L timeout -k 10 200 python3 -u tools/pose_sum_ab.py > $OUT/ab_$v.tmp 2>> $OUT/ab.err || exit 1
  sed "s/^/{\"lib\": \"$v\", \"r\": /; s/$/}/" $OUT/ab_$v.tmp >> $OUT/ab.jsonl
done
echo "exit=0"
