#!/bin/bash
# Round 4 final validation: the full GPU suite, smoke, the driver-shaped bench, genmove latency and the
# RL / value-generate drivers on the final tree.  Output: gpurun_out/r4_fin/
O=gpurun_out/r4_fin${FINTAG:-}
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step suite 600 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider --durations=10
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 240 python3 bench.py
step bench_d 240 python3 bench.py --gpus 1 --steps 20 --warmup 5
step genmove 240 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,16,32 --moves 4
