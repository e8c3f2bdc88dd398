set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02b; mkdir -p $OUT
make -j16 > $OUT/build.log 2>&1 &&
OSG_MATCH_PROFILE=1 timeout -k 10 120 python -u tools/latency_probe.py > $OUT/latency.jsonl 2> $OUT/latency.err &&
rm -f build/obj/pose.o && make -j16 POSE_PROF=1 > $OUT/build2.log 2>&1 &&
timeout -k 10 120 python -u tools/latency_probe.py > $OUT/latency_poseprof.jsonl 2>> $OUT/latency.err &&
timeout -k 10 120 python -u tools/pose_prof.py > $OUT/pose_prof.jsonl 2>> $OUT/latency.err
echo "exit=$?"
