#!/bin/bash
# Round 4 batch RP: host profile of the 20-game RL iteration (native lock-step driver).
O=gpurun_out/r4_rp
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step rlprof 400 python3 -u scripts/r4/pyprofile.py $O/rl20_cprofile.txt benchmarks/rl_iteration_benchmark.py --games 20 --iterations 2 --records device --drivers native
