#!/bin/bash
# A/B of bench stages between the current library and another build (OSG_LIB_PATH), alternating, two
# runs each (one gpurun call).  Usage: gpu_lib_ab.sh OUTDIR STAGES [OTHER_LIB]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03libab}
STAGES=$2
OTHER=${3:-$R/build/old/liborbslam3_amd.so}
mkdir -p $OUT
cd $R
for v in cur other cur other; do
  if [ $v = other ]; then export OSG_LIB_PATH=$OTHER; else unset OSG_LIB_PATH; fi
  timeout -k 10 300 python3 bench.py --no-cpu --no-stream --steps 3 --warmup 1 --only $STAGES > $OUT/$v.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1])
for k in '$STAGES'.split(','):
    x=d.get(k, {}); print('$v', k, x.get('value'), x.get('kernel_us_per_frame'), x.get('one_thread_frames_per_s'), x.get('wall_frames_per_s_incl_host_roundtrip'))
" >> $OUT/ab.txt
done
echo "exit=$?"
