#!/bin/bash
# Round-3 PMC passes and the final bench line (one gpurun call; the kernel trace and the VALU pass come
# from gpu_profile_r03.sh): FETCH_SIZE / WRITE_SIZE of the headline and stream kernels
# (-> pmc_traffic.json), the LBA engine's SQ / MFMA / HBM passes (-> r03_schur_pmc.json), then the bench
# line with those files.  Counters are never combined with traces; every GPU step has its own time
# limit and the chain stops at the first failure.  A heartbeat file keeps the call visibly alive.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03prof}
VALU_JSON=${2:-$R/profiles/r03_top2_valu_pmc.json}
mkdir -p $OUT
( while true; do date >> $OUT/heartbeat; sleep 30; done ) &
HB=$!
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES"
TRAF="--no-cpu --no-ba --no-gba --no-frames --steps 20 --warmup 5"
cd /tmp &&
echo fetch > $OUT/progress &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $TRAF > $OUT/fetch.log 2>&1 &&
echo write > $OUT/progress &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $TRAF > $OUT/write.log 2>&1 &&
python3 $R/tools/pmc_traffic.py $(find $OUT/fetch -name '*counter_collection.csv' | head -1) $(find $OUT/write -name '*counter_collection.csv' | head -1) $OUT/pmc_traffic.json &&
echo lba > $OUT/progress &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/lba_sq -o sq -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_sq.log 2>&1 &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/lba_fetch -o f -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_fetch.log 2>&1 &&
TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/lba_write -o w -- python3 $R/tools/lba_batch_bench.py > $OUT/lba_write.log 2>&1 &&
python3 $R/tools/pmc_kernel_summary.py $OUT/r03_schur_pmc.json $(find $OUT/lba_sq -name '*counter_collection.csv' | head -1) $(find $OUT/lba_fetch -name '*counter_collection.csv' | head -1) $(find $OUT/lba_write -name '*counter_collection.csv' | head -1) &&
echo bench > $OUT/progress &&
timeout -k 10 400 python3 $R/bench.py --traffic $OUT/pmc_traffic.json --valu-pmc $VALU_JSON --schur-pmc $OUT/r03_schur_pmc.json > $OUT/bench.json 2> $OUT/bench.err
rc=$?
kill $HB
echo "exit=$rc"
