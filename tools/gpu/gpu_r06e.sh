#!/bin/bash
# r06: why the compact-factor Schur kernel is slower: SQ wait / active breakdown and HBM traffic of every LBA
# kernel, compact (default) and whole-Hpl (OSG_LBA_HPL=1), over tools/lba_batch_bench.py (64 C4 windows, one
# thread).  Separate counter-only passes, each under its own time limit.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06e}
mkdir -p $OUT
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES"
SQ2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
cd /tmp
for mode in compact full; do
  if [ $mode = full ]; then export OSG_LBA_HPL=1; else unset OSG_LBA_HPL; fi
  TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc $SQ1 --output-format csv -d $OUT/$mode/sq1 -o sq1 -- python3 $R/tools/lba_batch_bench.py > $OUT/$mode.sq1.log 2>&1 || exit 1
  TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT/$mode/sq2 -o sq2 -- python3 $R/tools/lba_batch_bench.py > $OUT/$mode.sq2.log 2>&1 || exit 1
  TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$mode/f -o f -- python3 $R/tools/lba_batch_bench.py > $OUT/$mode.f.log 2>&1 || exit 1
  TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$mode/w -o w -- python3 $R/tools/lba_batch_bench.py > $OUT/$mode.w.log 2>&1 || exit 1
  python3 $R/tools/pmc_kernel_summary.py $OUT/lba_pmc_$mode.json $(find $OUT/$mode/sq1 -name '*counter_collection.csv' | head -1) $(find $OUT/$mode/f -name '*counter_collection.csv' | head -1) $(find $OUT/$mode/w -name '*counter_collection.csv' | head -1) > /dev/null || exit 1
  python3 $R/tools/pmc_kernel_summary.py $OUT/lba_pmc2_$mode.json $(find $OUT/$mode/sq2 -name '*counter_collection.csv' | head -1) > /dev/null || exit 1
  rm -rf $OUT/$mode
done
echo "exit=0"
