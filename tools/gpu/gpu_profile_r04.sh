#!/bin/bash
# Round-4 profiles (one gpurun call): the LBA engine's SQ / MFMA / FETCH_SIZE / WRITE_SIZE passes over
# tools/lba_batch_bench.py (64 C4 windows; separate runs, no counters combined with traces) ->
# r04_schur_pmc.json, then the kernel trace + stats of the default bench reading that file.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04prof}
mkdir -p $OUT
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES"
cd /tmp &&
echo lba > $OUT/progress &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/lba_sq -o sq -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_sq.log 2>&1 &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/lba_fetch -o f -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_fetch.log 2>&1 &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/lba_write -o w -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_write.log 2>&1 &&
python3 $R/tools/pmc_kernel_summary.py $OUT/r04_schur_pmc.json $(find $OUT/lba_sq -name '*counter_collection.csv' | head -1) $(find $OUT/lba_fetch -name '*counter_collection.csv' | head -1) $(find $OUT/lba_write -name '*counter_collection.csv' | head -1) > $OUT/schur_pmc_summary.txt &&
echo trace > $OUT/progress &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --no-wall --schur-pmc $OUT/r04_schur_pmc.json > $OUT/bench_under_trace.json 2> $OUT/trace.err
echo "exit=$?"
