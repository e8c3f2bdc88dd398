#!/bin/bash
# rocprofv3 over the headline kernel (tools/top2_batch_run.py): kernel trace + stats, then counter
# passes (instruction mix, MFMA busy, LDS, waits; HBM bytes).  Counters only in the --pmc passes, each
# pass under its own time limit.  Usage: tools/gpu/top2_pmc.sh OUTDIR [extra env assignments...]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-top2_pmc}; mkdir -p $OUT
C1=${C1:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"}
C2=${C2:-"SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"}
C3=${C3:-""}
cd /tmp &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/tools/top2_batch_run.py > $OUT/trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv -d $OUT/c1 -o c1 -- python3 $R/tools/top2_batch_run.py > $OUT/c1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv -d $OUT/c2 -o c2 -- python3 $R/tools/top2_batch_run.py > $OUT/c2.log 2>&1 &&
{ [ -z "$C3" ] || timeout -s KILL 90 rocprofv3 --pmc $C3 --output-format csv -d $OUT/c3 -o c3 -- python3 $R/tools/top2_batch_run.py > $OUT/c3.log 2>&1; } &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/tools/top2_batch_run.py > $OUT/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/tools/top2_batch_run.py > $OUT/write.log 2>&1
echo "exit=$?"
