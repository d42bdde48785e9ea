#!/bin/bash
# Round 4 batch D: fp8 value-trainer diagnosis (scripts/r4/fp8_diag.py), then the throughput
# benchmarks of batch B that do not depend on it.  Output: gpurun_out/r4_d/
O=gpurun_out/r4_d
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step diag_random 200 python3 -u scripts/r4/fp8_diag.py --planes random
step diag_games 200 python3 -u scripts/r4/fp8_diag.py --planes games
step diag_random_l4 200 python3 -u scripts/r4/fp8_diag.py --planes random --layers 4 --batch 32
step rl 500 python3 -u benchmarks/rl_iteration_benchmark.py --games 20,512 --iterations 1 --records device
step vgen 400 python3 -u benchmarks/value_generate_benchmark.py --games 256
