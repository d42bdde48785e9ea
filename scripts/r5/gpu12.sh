#!/bin/bash
# PMC passes on the weight-stationary conv (B = 16, 192 channels) vs the automatic tile; full GPU suite;
# SL bench at B = 8 / 16
O=gpurun_out/r5/b12
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
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
cat $O/pmc_summary.txt
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step sl16 300 python -u bench.py --batch 16 --steps 30 --warmup 5
step sl8 300 python -u bench.py --batch 8 --steps 30 --warmup 5
