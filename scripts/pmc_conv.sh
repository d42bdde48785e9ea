#!/bin/bash
# PMC counters for the conv kernels (kernel-trace only, no sys/runtime trace).
set -e
export PYTHONPATH=$PWD
OUT=gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for k in fwd dgrad wgrad; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python scripts/lab/kbench_one.py $k > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS -- python scripts/lab/kbench_one.py $k > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -- python scripts/lab/kbench_one.py $k > /dev/null 2>&1 || true
done
find $OUT -name "*counter_collection*" | head -20
