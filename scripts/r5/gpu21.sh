#!/bin/bash
# WS automatic up to B = 32: trainer tests, SL sweep, forward latency, B = 16 step profile
O=gpurun_out/r5/b21
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step tr_test 600 python -u -m pytest tests/test_hip_trainer.py tests/test_determinism_gpu.py tests/test_fp8_inference.py tests/test_gpu_features.py -x -q --timeout 300 --timeout-method thread
grep -E "passed|failed" $O/tr_test.log | tail -2
for B in 16 32 64; do
  step sl$B 300 python -u bench.py --batch $B --steps 200 --warmup 20
done
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32,64 --iters 30
grep bf16 $O/fwd_lat.log
prof prof_sl16 300 40 --batch 16 --steps 40 --warmup 10
