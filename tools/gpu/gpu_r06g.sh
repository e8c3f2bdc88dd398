#!/bin/bash
# r06: compact factor v5 (column-per-lane gathers) A/B (LBA tests + batch bench), then its FETCH / WRITE passes
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06g}; mkdir -p $OUT
bash tools/gpu/gpu_r06b.sh ${1:-r06g} || exit 1
cd /tmp
TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o f -- python3 $R/tools/lba_batch_bench.py > $OUT/f.log 2>&1 &&
TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o w -- python3 $R/tools/lba_batch_bench.py > $OUT/w.log 2>&1 &&
TS=1 BS=64 REPS=1 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/sq -o sq -- python3 $R/tools/lba_batch_bench.py > $OUT/sq.log 2>&1 &&
python3 $R/tools/pmc_kernel_summary.py $OUT/lba_pmc.json $(find $OUT/sq -name '*counter_collection.csv' | head -1) $(find $OUT/f -name '*counter_collection.csv' | head -1) $(find $OUT/w -name '*counter_collection.csv' | head -1) > /dev/null
rc=$?; rm -rf $OUT/f $OUT/w $OUT/sq; echo "exit=$rc"; exit $rc
