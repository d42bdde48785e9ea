#!/bin/bash
# Round 4 batch GP: host profile of the single-tree genmove (32 leaves per batch).
O=gpurun_out/r4_gp
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step genprof 300 python3 -u scripts/r4/genmove_profile.py $O/genmove_cprofile.txt --leaves 32 --moves 4
