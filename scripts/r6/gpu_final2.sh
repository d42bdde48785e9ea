#!/bin/bash
# Round-6 final tree (after the dual-wgrad revert and the RL / launcher changes): GPU suite, smoke(),
# the driver's bench command, the driver's 2-GPU form refused on a 1-GPU box.
O=gpurun_out/r6/final2
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_gpus2_on_1gpu 120 python bench.py --gpus 2 --steps 2 --warmup 1
grep -h '"value"' $O/bench1.log | cut -c1-200
tail -n 3 $O/bench_gpus2_on_1gpu.log
