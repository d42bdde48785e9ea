#!/bin/bash
# Round 4 batch V: narrow-N small-batch tiles 39 / 42 (tests; graph-timed per-layer forward at B = 1..64).
O=gpurun_out/r4_v
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
# step tests 300 python3 -u -m pytest tests/test_hip_kernels.py -k "tile_variants or ring_5x5" -m gpu -q --timeout 150 --timeout-method thread
step tiles 300 python3 -u scripts/r4/small_tile_graph_bench.py 1 4 16 64 256
