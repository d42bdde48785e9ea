#!/bin/bash
# Round 5 batch 6: first-layer wgrad in 96-wide halves (AGK_WGRAD0_HALF) A/B, reduce with 8 loads in flight
O=gpurun_out/r5/b6
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
source scripts/r5/lib.sh
step kt_half1 300 env AGK_WGRAD0_HALF=1 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -x -q --timeout 120 --timeout-method thread -k "wgrad or reduce or grads_match or trainer"
step kt_half0 300 env AGK_WGRAD0_HALF=0 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad or reduce"
for r in 1 2; do
  for h in 1 0; do
    step bench_half${h}_$r 300 env AGK_WGRAD0_HALF=$h python -u bench.py --steps 40 --warmup 5
  done
done
AGK_WGRAD0_HALF=1 prof trace_half1 300 10 --steps 10 --warmup 5 --min-warmup-s 0
AGK_WGRAD0_HALF=0 prof trace_half0 300 10 --steps 10 --warmup 5 --min-warmup-s 0
