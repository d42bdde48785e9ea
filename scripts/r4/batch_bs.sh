#!/bin/bash
# Round 4 batch BS: per-GPU batch of the headline bench, alternating on one box.
O=gpurun_out/r4_bs
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for r in 1 2; do
  for B in 2176 3264 4352; do
    step b${B}_r$r 240 python3 bench.py --batch $B --steps 40 --warmup 5
  done
done
