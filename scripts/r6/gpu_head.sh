#!/bin/bash
# Register-resident policy head: its tests, the driver's bench command, B = 16, and the step timeline.
O=gpurun_out/r6/head
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step tests 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step b16 300 python bench.py --gpus 1 --batch 16 --steps 300 --warmup 50
prof prof_b2176 300 5 --steps 10 --warmup 5
grep -h '"value"' $O/bench*.log $O/b16.log | cut -c1-200
