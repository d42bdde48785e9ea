#!/bin/bash
# Round 4 batch X: tile 42 vs the automatic tile at inference batches 32..362.
O=gpurun_out/r4_x
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
export TILES=0,64,128,42
step tiles 300 python3 -u scripts/r4/small_tile_graph_bench.py 32 48 64 96 128 192 256 362
