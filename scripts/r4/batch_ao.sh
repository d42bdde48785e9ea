#!/bin/bash
# Round 4 batch AO: automatic wgrad/dgrad overlap at small batches -- trainer tests, SL bench defaults.
O=gpurun_out/r4_ao
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 400 python3 -u -m pytest tests/test_hip_trainer.py tests/test_determinism_gpu.py tests/test_fp8_inference.py tests/test_rl_value.py tests/test_distributed_gpu.py -m gpu -q --timeout 150 --timeout-method thread
step sl16 120 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192
step sl256 120 python3 bench.py --batch 256 --steps 100 --warmup 20 --pool 8192
step bench 240 python3 bench.py --gpus 1 --steps 20 --warmup 5
