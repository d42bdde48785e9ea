#!/bin/bash
# memory-pipeline stall counters of the forward conv tile variants given as arguments
set -e
export PYTHONPATH=$PWD
OUT=gpurun_out/pmcfifo
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for t in ${@:-384 6}; do
  export ALPHAGO_AMD_CONV_TILE=$t
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$t/p1 --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- python scripts/lab/kbench_one.py fwd > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$t/p2 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -- python scripts/lab/kbench_one.py fwd > /dev/null 2>&1 || true
done
python scripts/pmc_summary.py $OUT 2>&1 | tail -60 || true
