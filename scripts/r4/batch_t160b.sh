#!/bin/bash
# Round 4 batch T160B: the automatic 32-pixel tile at the value width -- value/trainer tests, forward times.
O=gpurun_out/r4_t160b
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_conv160.py tests/test_rl_value.py tests/test_fp8_inference.py tests/test_hip_trainer.py -m gpu -q --timeout 150 --timeout-method thread
step fwd 200 python3 benchmarks/forward_latency_benchmark.py --batches 1,8,16,32
