#!/bin/bash
# pack_input writes the fp8 trunk's e4m3 input copy (no quantize_fp8 pass).
O=gpurun_out/r6/x8
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step tests 600 python -u -m pytest tests/test_hip_kernels.py tests/test_fp8_inference.py tests/test_hip_trainer.py -m gpu -x -q --timeout 120 --timeout-method thread
step value_fp8_r1 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
step value_fp8_r2 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
step sl_fp8 300 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
grep -h '"value"' $O/value_*.log $O/sl_fp8.log $O/bench1.log | cut -c1-200
