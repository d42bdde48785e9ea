#!/bin/bash
# Round 4 batch OV: wgrad on a side stream (--overlap) at small SL batches.
O=gpurun_out/r4_ov2
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for r in 1; do
  for B in 128 256 512 1024; do
    for OV in 0 1; do
      step sl${B}_ov${OV}_r$r 120 python3 bench.py --batch $B --steps 100 --warmup 20 --pool 8192 $([ $OV = 1 ] && echo --overlap)
    done
  done
done
