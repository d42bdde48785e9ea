#!/bin/bash
# Last check of the shipped tree: GPU suite, smoke(), the driver's bench command.
O=gpurun_out/r6/last2
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step value_fp8 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
grep -h '"value"' $O/bench1.log $O/value_fp8.log | cut -c1-200
