#!/bin/bash
# Round 4 batch G: value-net precision parity on the value-teacher task (4 epochs, fp32 / bf16 / fp8 /
# fp8-forward arms).  Output: gpurun_out/r4_g/
O=gpurun_out/r4_g
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step value_parity 1100 python3 -u scripts/value_fp8_parity.py $O/value_parity.json --positions 32768 --epochs 4 --arms torch-fp32,hip-bf16,hip-fp8,hip-fp8fwd
