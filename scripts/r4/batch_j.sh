#!/bin/bash
# Round 4 batch J: the compact-halo lab forward/dgrad (lab tile 5, 6) inside the power-limited training
# step (ALPHAGO_AMD_LAB_TILE), interleaved same-box A/B + trace.  Output: gpurun_out/r4_j/
O=gpurun_out/r4_j
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
ab() { step ab_lab$1_$RANDOM 200 env ALPHAGO_AMD_LAB_TILE=$1 python3 bench.py --steps 100 --warmup 20; }
ab 0; ab 5; ab 6; ab 0; ab 5; ab 6
ALPHAGO_AMD_LAB_TILE=5 prof prof5 300 5 --steps 20 --warmup 5
