#!/bin/bash
# r06: k_schur_rows_c's per-workgroup timeline (make SR_PROF=1 build in build/srprof), graph 0 of a 64-window batch
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06o}; mkdir -p $OUT
OSG_LIB_PATH=$PWD/build/srprof/liborbslam3_amd.so OSG_SR_PROF_OUT=$OUT/sr.bin TS=1 BS=64 REPS=1 timeout -k 10 200 python -u tools/lba_batch_bench.py > $OUT/bench.txt 2>&1 &&
python3 tools/sr_prof.py $OUT/sr.bin > $OUT/sr.txt 2>&1
rc=$?; echo "exit=$rc"; exit $rc
