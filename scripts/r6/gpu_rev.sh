#!/bin/bash
# Policy head over the boards in reverse order (Infinity Cache residency of the last-written boards).
O=gpurun_out/r6/rev
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step tests 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -m gpu -x -q --timeout 120 --timeout-method thread -k "head or bce or step"
prof prof_b2176 300 5 --steps 10 --warmup 5
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5
grep -h '"value"' $O/bench*.log | cut -c1-200
