#!/bin/bash
# Global BA A/B between the current library and another build (OSG_LIB_PATH), two runs each (one gpurun call).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03gbaab}
OTHER=${2:-$R/build/old/liborbslam3_amd.so}
mkdir -p $OUT
cd $R
ARGS="--no-cpu --no-stream --no-ba --no-frames --no-gba-map --steps 3 --warmup 1"
for v in cur other cur other; do
  if [ $v = other ]; then export OSG_LIB_PATH=$OTHER; else unset OSG_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py $ARGS > $OUT/$v.json 2>> $OUT/err.log || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); g=d['global_ba']; print('$v', g['value'], g['ms_per_gba'])" >> $OUT/ab.txt
done
echo "exit=$?"
