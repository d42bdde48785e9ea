#!/bin/bash
O=gpurun_out/r6/e5
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step tests 600 python -u -m pytest tests/test_fp8_inference.py tests/test_hip_trainer.py tests/test_hip_kernels.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
