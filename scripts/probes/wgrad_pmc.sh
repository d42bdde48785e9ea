#!/bin/bash
# PMC passes (one counter group per run) on the production wgrad kernels: 3x3 192x192 and layer 0.
set -e
export PYTHONPATH=$PWD TMPDIR=/tmp
OUT=${OUT:-gpurun_out/wpmc}
mkdir -p $OUT
for k in w3 w0; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python3 scripts/probes/wgrad_pmc_one.py $k > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS -- python3 scripts/probes/wgrad_pmc_one.py $k > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -- python3 scripts/probes/wgrad_pmc_one.py $k > /dev/null 2>&1 || true
done
python3 scripts/pmc_summary.py $OUT
