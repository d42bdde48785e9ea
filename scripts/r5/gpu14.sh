#!/bin/bash
# weight-stationary: slice-set XCD placement (k auto / 1 / 2 / 4), distinct per-layer weights
O=gpurun_out/r5/b14
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step ws_test 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "weight_stationary"
grep -q " passed" $O/ws_test.log && ! grep -q "failed" $O/ws_test.log || exit 1
for k in 0 1 2 4; do
  step ws_bench_k$k 300 env AGK_WS_K=$k WS_BATCHES=1,4,8,16,32 python -u scripts/r5/ws_bench.py
  grep '"C"' $O/ws_bench_k$k.log
done
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32 --iters 30
grep bf16 $O/fwd_lat.log
