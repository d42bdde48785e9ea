#!/bin/bash
# weight-stationary v2 (epilogue waves, 2-deep prefetch, XCD order): tests, per-layer times, PMC, latency
O=gpurun_out/r5/b13
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step ws_test 300 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -x -q --timeout 120 --timeout-method thread -k "weight_stationary or splitk"
grep -E "passed|failed" $O/ws_test.log | tail -2
grep -q " passed" $O/ws_test.log && ! grep -q "failed" $O/ws_test.log || exit 1
step ws_bench 300 python -u scripts/r5/ws_bench.py
grep '"C"' $O/ws_bench.log
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/pmc/p$i --pmc $P -- python3 scripts/r5/ws_one.py 16 192 > $O/pmc_p$i.log 2>&1
  rc=$?; echo "[pmc p$i] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 scripts/r4/pmc_by_kernel.py $O/pmc > $O/pmc_summary.txt 2>&1
find $O/pmc -name "*kernel_trace.csv" -delete
grep -E "==|wait_any|mfma_busy|TCC_MISS" $O/pmc_summary.txt
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32 --iters 30
grep bf16 $O/fwd_lat.log
