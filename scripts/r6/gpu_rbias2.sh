#!/bin/bash
# Split-K reduce: the bias in its own blocks (4-way split order), off the slab blocks.
O=gpurun_out/r6/rbias2
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step tests 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py tests/test_determinism_gpu.py tests/test_conv160.py -m gpu -x -q --timeout 120 --timeout-method thread
prof prof_b2176 300 5 --steps 10 --warmup 5
prof prof16 300 50 --batch 16 --steps 300 --warmup 50
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b16_r1 120 python bench.py --gpus 1 --batch 16 --steps 300 --warmup 50
step b16_r2 120 python bench.py --gpus 1 --batch 16 --steps 300 --warmup 50
step b32 120 python bench.py --gpus 1 --batch 32 --steps 300 --warmup 50
step value_fp8 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
grep -h '"value"' $O/bench*.log $O/b16*.log $O/b32.log $O/value_fp8.log | cut -c1-200
