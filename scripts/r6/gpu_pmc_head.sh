#!/bin/bash
# HBM bytes per kernel of the SL step (policy head, pack, reduce): FETCH_SIZE and WRITE_SIZE in passes
# of their own (3 + 2 TCC counters), kernel trace only.
O=gpurun_out/r6/pmc
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/p1 --pmc FETCH_SIZE -- python bench.py --gpus 1 --steps 3 --warmup 2 --min-warmup-s 0 > $O/p1.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/p2 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -- python bench.py --gpus 1 --steps 3 --warmup 2 --min-warmup-s 0 > $O/p2.log 2>&1
rc=$?
python3 scripts/r4/pmc_by_kernel.py $O > $O/pmc_summary.txt 2>&1
find $O -name "*kernel_trace.csv" -delete
find $O -name "*counter_collection.csv" -size +20M -delete
grep -A4 "policy_head\|pack_input\|reduce_kernel" $O/pmc_summary.txt | head -40
exit $rc
