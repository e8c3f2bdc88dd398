#!/bin/bash
# Global-BA A/B: tools/gba_kernel_probe.py with the current library and build/old (OSG_LIB_PATH),
# alternating, two runs each.  Each GPU step has its own time limit; the chain stops at a failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-gbaab}
mkdir -p $OUT
cd $R
for v in cur old cur old; do
  if [ $v = old ]; then export OSG_LIB_PATH=$R/build/old/liborbslam3_amd.so; else unset OSG_LIB_PATH; fi
  timeout -k 10 240 python3 -u tools/gba_kernel_probe.py --label $v >> $OUT/ab.jsonl 2>> $OUT/err.log || exit 1
done
echo "exit=0"
