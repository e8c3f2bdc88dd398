#!/bin/bash
# Global BA: the compact per-block factor (default) against the whole-Hpl form (OSG_LBA_HPL=1), alternating
# processes (the switch is read once per process).  Each run under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06gba}
mkdir -p $OUT
cd $R
for rep in 0 1; do
  timeout -k 10 240 env OSG_LBA_HPL=0 python3 -u tools/gba_kernel_probe.py --label compact >> $OUT/gba.jsonl 2>> $OUT/gba.err || exit 1
  timeout -k 10 240 env OSG_LBA_HPL=1 python3 -u tools/gba_kernel_probe.py --label hpl >> $OUT/gba.jsonl 2>> $OUT/gba.err || exit 1
done
python3 -c "
import json
for l in open('$OUT/gba.jsonl'):
    d=json.loads(l); k=d['kernel_ms']; top=sorted(k.items(), key=lambda x:-x[1])[:6]
    print(d['label'], d['map'], d['ms_per_call'], d['iterations'], d['trials'], top)"
