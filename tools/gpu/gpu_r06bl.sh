#!/bin/bash
# k_chol_back_large Linv prefetch: the GBA tests (incl. OSG_BACKL_PRE bit identity), then the GBA probe alternating
# OSG_BACKL_PRE=0/1 in separate processes.  Each GPU step time-limited; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06bs}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gba" > $OUT/pytest_gba.log 2>&1 || { echo "gba tests failed"; tail -30 $OUT/pytest_gba.log; exit 1; }
tail -2 $OUT/pytest_gba.log
for rep in 0 1; do
  timeout -k 10 240 env OSG_BACKL_PRE=0 python3 -u tools/gba_kernel_probe.py --label pre0 >> $OUT/gba.jsonl 2>> $OUT/gba.err || exit 1
  timeout -k 10 240 env OSG_BACKL_PRE=1 python3 -u tools/gba_kernel_probe.py --label pre1 >> $OUT/gba.jsonl 2>> $OUT/gba.err || exit 1
done
python3 -c "
import json
for l in open('$OUT/gba.jsonl'):
    d=json.loads(l); k=d['kernel_ms']
    print(d['label'], d['map'], d['ms_per_call'], d['iterations'], d['trials'], 'chol', k.get('chol'), 'chol_back', k.get('chol_back'))"
