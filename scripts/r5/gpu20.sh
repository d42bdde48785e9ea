#!/bin/bash
# weight-stationary with the WS weight order + LDS row ring: tests, per-layer times, suite, SL sweep, latency
O=gpurun_out/r5/b20
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step ws_test 300 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -x -q --timeout 120 --timeout-method thread -k "weight_stationary or splitk"
grep -E "passed|failed" $O/ws_test.log | tail -2
grep -q " passed" $O/ws_test.log && ! grep -q "failed" $O/ws_test.log || exit 1
step ws_bench 300 env WS_BATCHES=1,4,8,16,32,64 python -u scripts/r5/ws_bench.py
grep '"C"' $O/ws_bench.log
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -E "passed|failed" $O/suite.log | tail -2
for B in 1 8 16; do
  step sl$B 300 python -u bench.py --batch $B --steps 200 --warmup 20
done
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32 --iters 30
grep bf16 $O/fwd_lat.log
