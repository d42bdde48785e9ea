#!/bin/bash
# Round-6 batch 7: value precision parity with the unguarded fp8 scale (the default again), 4x positions.
O=gpurun_out/r6/fp8
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 620 python -u scripts/value_fp8_parity.py $O/parity_value_4x_noguard.json --task material \
  --positions 262144 --epochs 4 --arms torch-fp32,hip-bf16,hip-fp8 --optimizer adam --lr 0.0003 --decay 0.005 \
  --seeds 5 > $O/parity_value_4x_noguard.log 2>&1
rc=$?
grep "epoch 4" $O/parity_value_4x_noguard.log
exit $rc
