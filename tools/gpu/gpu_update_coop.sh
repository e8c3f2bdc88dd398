#!/bin/bash
# k_update with one thread per Hpl block (OSG_UPDATE_COOP=1): the bit-identity test, then the LocalBA stage
# alternating the two forms (kernel time per step from --detail).  Each GPU step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-upcoop}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "variants_bit_identical or lba_parity" > $OUT/pytest.log 2>&1 || { echo "tests failed"; exit 1; }
ARGS="--only local_ba --no-cpu --no-stream --steps 5 --warmup 2"
for v in 0 1 0 1; do
  OSG_UPDATE_COOP=$v timeout -k 10 240 python bench.py $ARGS --detail $OUT/lba_$v.json >> $OUT/lba_$v.jsonl 2>> $OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/lba_$v.json'));b=d['local_ba'];print('$v',b['value'],json.dumps(b['kernel_ms_per_step']))" >> $OUT/summary.txt || exit 1
done
echo "exit=0"
