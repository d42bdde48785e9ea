#!/bin/bash
# Round 4 batch PF: rocprofv3 kernel trace + stats of the SL step on the final tree (B = 2176 and 16).
O=gpurun_out/r4_pf
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
prof final_b2176 300 10 --steps 10 --warmup 5 --min-warmup-s 0
prof final_b16 300 50 --batch 16 --steps 50 --warmup 20 --min-warmup-s 0 --pool 4096
