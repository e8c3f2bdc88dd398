#!/bin/bash
# r06: the LBA engine's PMC passes on the final compact-factor kernels (SQ / MFMA, SQ waits, FETCH_SIZE,
# WRITE_SIZE; separate counter-only runs) over tools/lba_batch_bench.py (64 C4 windows, one thread)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06j}; mkdir -p $OUT
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES"
SQ2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
cd /tmp
TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc $SQ1 --output-format csv -d $OUT/sq1 -o sq1 -- python3 $R/tools/lba_batch_bench.py > $OUT/sq1.log 2>&1 &&
TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT/sq2 -o sq2 -- python3 $R/tools/lba_batch_bench.py > $OUT/sq2.log 2>&1 &&
TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o f -- python3 $R/tools/lba_batch_bench.py > $OUT/f.log 2>&1 &&
TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o w -- python3 $R/tools/lba_batch_bench.py > $OUT/w.log 2>&1 &&
python3 $R/tools/pmc_kernel_summary.py $OUT/lba_pmc.json $(find $OUT/sq1 -name '*counter_collection.csv' | head -1) $(find $OUT/f -name '*counter_collection.csv' | head -1) $(find $OUT/w -name '*counter_collection.csv' | head -1) > /dev/null &&
python3 $R/tools/pmc_kernel_summary.py $OUT/lba_pmc_waits.json $(find $OUT/sq2 -name '*counter_collection.csv' | head -1) > /dev/null
rc=$?; rm -rf $OUT/sq1 $OUT/sq2 $OUT/f $OUT/w; echo "exit=$rc"; exit $rc
