#!/bin/bash
# Round 4 batch MS: wgrad minimum stages per split (slab size vs split length) at small SL batches.
O=gpurun_out/r4_ms2
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for r in 1 2; do
  for MS in 2 4 6 8; do
    step sl16_ms${MS}_r$r 120 env ALPHAGO_AMD_WGRAD_MIN_STAGES=$MS python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192
  done
done
