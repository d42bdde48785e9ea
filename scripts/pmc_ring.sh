#!/bin/bash
# PMC comparison: gather (2-buffer) vs ring forward conv kernels.
set -e
export PYTHONPATH=$PWD
OUT=gpurun_out/pmc2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
for k in fwd fwdring; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python scripts/lab/kbench_one.py $k > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p2 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA -- python scripts/lab/kbench_one.py $k > /dev/null 2>&1 || true
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$k/p3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum -- python scripts/lab/kbench_one.py $k > /dev/null 2>&1 || true
done
python scripts/pmc_summary.py $OUT
