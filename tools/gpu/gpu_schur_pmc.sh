#!/bin/bash
# PMC passes over the LBA batch (k_schur_rows and the Cholesky MFMA kernels): instruction mix and
# MFMA busy cycles, FP64-MFMA (default) and VALU (OSG_SCHUR_VALU=1) Schur products.  Counters only,
# no traces; each pass under its own time limit.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-schur_pmc}; mkdir -p $OUT
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE"
make -j16 > $OUT/build.log 2>&1 && cd /tmp &&
KT= TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $OUT/mfma_c1 -o c1 -- python3 $R/tools/lba_batch_bench.py > $OUT/mfma_c1.log 2>&1 &&
KT= TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $OUT/mfma_c2 -o c2 -- python3 $R/tools/lba_batch_bench.py > $OUT/mfma_c2.log 2>&1 &&
OSG_SCHUR_VALU=1 TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $OUT/valu_c1 -o c1 -- python3 $R/tools/lba_batch_bench.py > $OUT/valu_c1.log 2>&1 &&
OSG_SCHUR_VALU=1 TS=1 BS=64 timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $OUT/valu_c2 -o c2 -- python3 $R/tools/lba_batch_bench.py > $OUT/valu_c2.log 2>&1
echo "exit=$?"
