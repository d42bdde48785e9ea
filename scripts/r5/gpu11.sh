#!/bin/bash
O=gpurun_out/r5/b11
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
source scripts/r5/lib.sh
step ws_test 300 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -x -q --timeout 120 --timeout-method thread -k "weight_stationary or splitk"
for w in 256 128 512; do
  step ws_bench_$w 300 env AGK_WS_WGS=$w python -u scripts/r5/ws_bench.py
  cat $O/ws_bench_$w.log | grep '"C"'
done
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32 --iters 30
grep bf16 $O/fwd_lat.log
