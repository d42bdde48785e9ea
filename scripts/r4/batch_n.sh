#!/bin/bash
# Round 4 batch N: value parity on the learnable configuration (as batch G2), PMC passes of the B = 16 step.
# Output: gpurun_out/r4_n/
O=gpurun_out/r4_n
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step value_parity 1000 python3 -u scripts/value_fp8_parity.py $O/value_parity.json --task teacher --init he --lr 0.01 --positions 32768 --heldout 8192 --epochs 16 --arms torch-fp32,hip-bf16,hip-fp8,hip-fp8fwd
step pmc16 400 bash scripts/r4/pmc_small.sh $O/pmc16 16
