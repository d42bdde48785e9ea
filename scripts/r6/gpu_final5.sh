#!/bin/bash
# Round-6 final tree (last: after the e4m3 input pack): GPU suite, smoke(), the
# driver's bench command twice, value training, B = 16, the 2-GPU form refused on a 1-GPU box.
O=gpurun_out/r6/final5
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step value_fp8 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
step value_bf16 300 python -u benchmarks/value_training_benchmark.py --precision bf16 --steps 30
step b16 300 python bench.py --gpus 1 --batch 16 --steps 300 --warmup 50
step bench_gpus2_on_1gpu 120 python bench.py --gpus 2 --steps 2 --warmup 1
grep -h '"value"' $O/bench1.log $O/bench2.log $O/b16.log | cut -c1-200
tail -n 3 $O/bench_gpus2_on_1gpu.log
