#!/bin/bash
# Round 4 batch EP: fp8 epilogue -- hoisted loads (see git log; new = this tree, old = the previous build), value
# training at B = 1024 and the fp8 value kernel tests, alternating builds on one box.
O=gpurun_out/r4_ep${EPTAG:-}
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
SO=alphago_amd/_hip_kernels.so
step tests 300 python3 -u -m pytest tests/test_fp8_inference.py tests/test_conv160.py tests/test_hip_kernels.py -k "fp8 or 160 or value or Fp8 or bf8" -m gpu -q --timeout 150 --timeout-method thread
for r in 1 2; do
  cp ab/_hip_kernels_new2.so $SO
  step value_new_r$r 200 python3 -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30 --warmup 10
  cp ab/_hip_kernels_old.so $SO
  step value_old_r$r 200 python3 -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30 --warmup 10
done
cp ab/_hip_kernels_new2.so $SO
step fwd_new 200 python3 benchmarks/forward_latency_benchmark.py --batches 256,1024
cp ab/_hip_kernels_old.so $SO
step fwd_old 200 python3 benchmarks/forward_latency_benchmark.py --batches 256,1024
cp ab/_hip_kernels_new2.so $SO
