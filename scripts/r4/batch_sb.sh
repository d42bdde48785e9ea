#!/bin/bash
# Round 4 batch SB: SL throughput across batch sizes on the final tree (defaults).
O=gpurun_out/r4_sb
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for B in 1 4 8 16 32 64 256 1024; do
  step sl_b$B 150 python3 bench.py --batch $B --steps 200 --warmup 30 --pool 8192
done
