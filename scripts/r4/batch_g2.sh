#!/bin/bash
# Round 4 batch G2: value-net precision parity on the value-teacher task with a He-initialised student
# (16 epochs, lr 0.01; the learnable configuration of the batch K / M sweeps).  Output: gpurun_out/r4_g2/
O=gpurun_out/r4_g2
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step value_parity 1100 python3 -u scripts/value_fp8_parity.py $O/value_parity.json --task teacher --init he --lr 0.01 --positions 32768 --heldout 8192 --epochs 16 --arms torch-fp32,hip-bf16,hip-fp8,hip-fp8fwd
