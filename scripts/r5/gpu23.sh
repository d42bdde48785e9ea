#!/bin/bash
# PMC of the weight-stationary conv (ring + WS order) at B = 16 vs the automatic tile; B = 16 forward trace
O=gpurun_out/r5/b23
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc/p$i --pmc $P -- python3 scripts/r5/ws_one.py 16 192 > $O/pmc_p$i.log 2>&1
  rc=$?; echo "[pmc p$i] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 scripts/r4/pmc_by_kernel.py $O/pmc > $O/pmc_summary.txt 2>&1
find $O/pmc -name "*kernel_trace.csv" -delete
grep -E "==|wait_any|mfma_busy|TCC_MISS|LDS_BANK" $O/pmc_summary.txt
