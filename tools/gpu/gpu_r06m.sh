#!/bin/bash
# r06: after k_schur_rows_c<2> became the default: the variant bit-identity tests and the full-size C5
# sharded test, then the LBA PMC passes (gpu_r06j.sh) on the new default
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06m}; mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_shard_dist.py -m gpu -x -v -k "variants_bit_identical or compact_factor or sharded" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 &&
bash tools/gpu/gpu_r06j.sh ${1:-r06m}
rc=$?; echo "exit=$rc"; exit $rc
