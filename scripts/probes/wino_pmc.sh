#!/bin/bash
# Kernel-lab Winograd forward vs the production 3x3 forward: PMC passes (B = 2176, 192 -> 192).
set -e
export PYTHONPATH=$PWD TMPDIR=/tmp
OUT=${OUT:-gpurun_out/winopmc}
mkdir -p $OUT
for k in wino:0 fwd:386; do
  d=$OUT/${k/:/_}
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $d/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python3 scripts/probes/conv_power_probe.py $k 1 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $d/p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_LDS -- python3 scripts/probes/conv_power_probe.py $k 1 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $d/p3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -- python3 scripts/probes/conv_power_probe.py $k 1 > /dev/null 2>&1 || true
  find $d -name "*kernel_trace.csv" -path "*p2*" -delete; find $d -name "*kernel_trace.csv" -path "*p3*" -delete
done
python3 scripts/pmc_summary.py $OUT
