#!/bin/bash
# Round-6 final tree: GPU suite, smoke(), the driver's bench command, value training, headline timeline.
O=gpurun_out/r6/final
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step value_fp8 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
step value_bf16 300 python -u benchmarks/value_training_benchmark.py --precision bf16 --steps 30
prof prof_b2176 300 5 --steps 10 --warmup 5
grep -h '"value"' $O/bench*.log | cut -c1-200
