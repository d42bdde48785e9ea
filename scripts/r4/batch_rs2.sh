#!/bin/bash
# Round 4 batch RS2: split-K wgrad reduce on a side stream at small SL batches.
O=gpurun_out/r4_rs2
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for r in 1 2; do
  for B in 16 64; do
    for RS in 0 1; do
      step sl${B}_rs${RS}_r$r 120 python3 bench.py --batch $B --steps 300 --warmup 50 --pool 8192 --reduce-stream $RS
    done
  done
done
