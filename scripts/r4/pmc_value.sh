#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) on the fp8 value-training step.
# Usage: scripts/r4/pmc_value.sh OUTDIR [value_training_benchmark args]
set -e
OUT=$1; shift 1
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p $OUT
ARGS="--steps 8 --warmup 3 --pool 8192 --heldout 1024 $@"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python3 benchmarks/value_training_benchmark.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -- python3 benchmarks/value_training_benchmark.py $ARGS > $OUT/p2.log 2>&1
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 --pmc TCC_HIT_sum TCC_MISS_sum -- python3 benchmarks/value_training_benchmark.py $ARGS > $OUT/p3.log 2>&1
python3 scripts/r4/pmc_by_kernel.py $OUT > $OUT/summary.txt
find $OUT -name "*kernel_trace.csv" -delete
cat $OUT/summary.txt
