#!/bin/bash
# Round 4 batch B: lock-step driver throughput (RL iteration, value-generate), value fp8 parity,
# genmove latency, value training speed.  Output: gpurun_out/r4_b/
O=gpurun_out/r4_b
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step value_fp8 200 python3 -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30 --warmup 10
step value_bf16 200 python3 -u benchmarks/value_training_benchmark.py --precision bf16 --steps 30 --warmup 10
step rl 500 python3 -u benchmarks/rl_iteration_benchmark.py --games 20,512 --iterations 1 --records device
step vgen 400 python3 -u benchmarks/value_generate_benchmark.py --games 256
step genmove 300 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,16,32 --moves 4
step value_parity 700 python3 -u scripts/value_fp8_parity.py $O/value_parity.json --positions 32768 --epochs 4 --arms torch-fp32,hip-bf16,hip-fp8,hip-fp8fwd
