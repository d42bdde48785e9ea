#!/bin/bash
# Round 4 batch AO2: automatic overlap at the split-K batches (B = 1 / 4 / 8 / 32), on vs off.
O=gpurun_out/r4_ao3
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for B in 2 4 4 6; do
  step sl${B}_auto_$RANDOM 120 python3 bench.py --batch $B --steps 300 --warmup 50 --pool 4096
  step sl${B}_off_$RANDOM 120 env ALPHAGO_AMD_OVERLAP=0 python3 bench.py --batch $B --steps 300 --warmup 50 --pool 4096
done
