#!/bin/bash
# Round 4 batch Z: split-K at the value width -- kernel / trainer tests, forward GPU time B = 1..64.
O=gpurun_out/r4_z
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py tests/test_conv160.py tests/test_fp8_inference.py -k "splitk or conv160 or 160 or small or bucket" -m gpu -q --timeout 150 --timeout-method thread
step fwd 200 python3 benchmarks/forward_latency_benchmark.py --batches 1,2,4,8,16,64
step fwd_nosk 200 env ALPHAGO_AMD_SPLITK=0 python3 benchmarks/forward_latency_benchmark.py --batches 1,2,4
