#!/bin/bash
# Round-6 batch 9: the torch fp32 arm of the self-play value run (same seeded dataset as batch 6: the
# value stage regenerates it and records its sha1).
RL_TAG=${RL_TAG:-_lr0.01}
O=gpurun_out/r6/ev
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step value_fp32 1100 python scripts/r6/evidence.py value $O --nets r6_nets --tag $RL_TAG --positions 204800 \
  --batch-games 4096 --epochs 6 --batch 256 --seeds 3 --arms torch-fp32
tail -3 $O/value_fp32.log
