#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) on the SL step at a small batch.
# Usage: scripts/r4/pmc_small.sh OUTDIR BATCH [bench args]
set -e
OUT=$1; B=$2; shift 2
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p $OUT
ARGS="--batch $B --steps 10 --warmup 3 --min-warmup-s 0 --pool 2048 $@"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 --pmc TCC_HIT_sum TCC_MISS_sum -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
python3 scripts/r4/pmc_by_kernel.py $OUT > $OUT/summary.txt
find $OUT -name "*kernel_trace.csv" -delete
cat $OUT/summary.txt
