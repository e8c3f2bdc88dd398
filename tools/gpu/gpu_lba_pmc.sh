#!/bin/bash
# The LBA engine's PMC passes (SQ / MFMA, FETCH_SIZE, WRITE_SIZE; separate runs, counters only, no
# traces) over tools/lba_batch_bench.py (64 C4 windows) -> OUT/lba_pmc.json (per kernel, the
# bench's --schur-pmc input).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-lba_pmc}
mkdir -p $OUT
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES"
cd /tmp &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/lba_sq -o sq -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_sq.log 2>&1 &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/lba_fetch -o f -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_fetch.log 2>&1 &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/lba_write -o w -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_write.log 2>&1 &&
python3 $R/tools/pmc_kernel_summary.py $OUT/lba_pmc.json $(find $OUT/lba_sq -name '*counter_collection.csv' | head -1) $(find $OUT/lba_fetch -name '*counter_collection.csv' | head -1) $(find $OUT/lba_write -name '*counter_collection.csv' | head -1) > $OUT/pmc_summary.txt
rc=$?; echo "exit=$rc"; exit $rc
