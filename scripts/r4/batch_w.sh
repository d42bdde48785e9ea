#!/bin/bash
# Round 4 batch W: launch floor of graph chains, split-K sweep at B = 1..4, tile 42 at large batches.
O=gpurun_out/r4_w
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step floor 300 python3 -u scripts/r4/launch_floor.py
