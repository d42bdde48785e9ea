#!/bin/bash
# MFMA utilisation per kernel of the final SL step (B = 2176): one SQ/GRBM counter pass, kernel trace only.
O=gpurun_out/r6/pmc_mfma
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/p1 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -- python bench.py --gpus 1 --steps 3 --warmup 2 --min-warmup-s 0 > $O/p1.log 2>&1
rc=$?
python3 scripts/r4/pmc_by_kernel.py $O > $O/pmc_summary.txt 2>&1
find $O -name "*kernel_trace.csv" -delete
find $O -name "*counter_collection.csv" -size +20M -delete
grep -A12 "conv_fwd_kernel<192, 0\|conv_fwd_kernel<192, 3\|conv_wgrad_kernel<192, 192\|conv_wgrad_kernel<96" $O/pmc_summary.txt | grep "==\|mfma_busy\|wait_any" | head -20
exit $rc
