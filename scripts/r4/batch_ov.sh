#!/bin/bash
# Round 4 batch OV: wgrad on a side stream (--overlap) at small SL batches.
O=gpurun_out/r4_ov
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for r in 1 2; do
  for B in 16 64; do
    for OV in 0 1; do
      step sl${B}_ov${OV}_r$r 120 python3 bench.py --batch $B --steps 300 --warmup 50 --pool 8192 $([ $OV = 1 ] && echo --overlap)
    done
  done
done
