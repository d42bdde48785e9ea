#!/bin/bash
# PMC counters of the forward conv for the tile variants given as arguments (default: 384 4)
set -e
export PYTHONPATH=$PWD
OUT=gpurun_out/pmcfwd
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for t in ${@:-384 4}; do
  export ALPHAGO_AMD_CONV_TILE=$t
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$t/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python scripts/lab/kbench_one.py ${WHICH:-fwd} > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$t/p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS -- python scripts/lab/kbench_one.py ${WHICH:-fwd} > /dev/null 2>&1
done
python scripts/pmc_summary.py $OUT 2>&1 | tail -60 || true
