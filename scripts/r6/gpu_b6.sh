#!/bin/bash
# Round-6 batch 6: value net on self-play outcomes (value-generate procedure with the SL net and its RL
# fine-tune RL_TAG, >= 200k positions; train-value defaults in HIP bf16 / HIP fp8 x 3 seeds, torch fp32
# seed 0), then search with that value net vs the greedy raw SL policy.
RL_TAG=${RL_TAG:-_lr0.003}
O=gpurun_out/r6/ev
mkdir -p $O gpurun_out/r6/nets
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step value_hip 900 python scripts/r6/evidence.py value $O --nets r6_nets --tag $RL_TAG --positions 204800 \
  --batch-games 4096 --epochs 6 --batch 256 --seeds 3 --arms hip-bf16,hip-fp8
cp r6_nets/value.* gpurun_out/r6/nets/ 2>/dev/null
step search 600 python scripts/r6/evidence.py search $O --nets r6_nets --games 200 --playouts 1600 --leaves 32
tail -3 $O/value_hip.log $O/search.log
