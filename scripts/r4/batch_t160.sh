#!/bin/bash
# Round 4 batch T160: a 32-pixel tile for the 160-wide value layers (tests; graph-timed per-layer
# forward at the value width vs tile 64 / split-K).
O=gpurun_out/r4_t160
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_conv160.py -m gpu -q --timeout 150 --timeout-method thread
export WIDTH=160 TILES=64,36,38
step tiles 300 python3 -u scripts/r4/small_tile_graph_bench.py 1 4 8 16 32 45 64
