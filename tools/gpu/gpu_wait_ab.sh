#!/bin/bash
# osg_wait A/B: the polled event (default) against OSG_WAIT=sync, alternating, on bench stages and the
# single-call latency probe (one gpurun call).  Usage: gpu_wait_ab.sh OUTDIR STAGES
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03waitab}
STAGES=$2
mkdir -p $OUT
cd $R
for v in spin sync spin sync; do
  if [ $v = sync ]; then export OSG_WAIT=sync; else unset OSG_WAIT; fi
  timeout -k 10 300 python3 bench.py --no-cpu --no-stream --steps 3 --warmup 1 --only $STAGES > $OUT/$v.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1])
for k in '$STAGES'.split(','):
    x=d.get(k, {}); print('$v', k, x.get('value'), x.get('kernel_us_per_frame'), x.get('one_thread_frames_per_s'), x.get('wall_frames_per_s_incl_host_roundtrip'))
" >> $OUT/ab.txt
  timeout -k 10 200 python3 tools/latency_probe.py 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    for k,v in d.items():
        if 'wall_us' in v: print('$v', k, v['wall_us'], v['kernel_us'])
        else: print('$v', k, {kk: (vv['wall_us'], vv['kernel_us']) for kk, vv in v.items()})
" >> $OUT/ab.txt || exit 1
done
echo "exit=$?"
