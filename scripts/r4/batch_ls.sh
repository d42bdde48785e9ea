#!/bin/bash
# Round 4 batch LS: lock-step host trims (mask-mode sampling kernel, cached numpy views and events) --
# tests, RL iteration at 20 / 512 games, value-generate.
O=gpurun_out/r4_ls
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_lockstep.py tests/test_rl_value.py -k "sample_moves or lockstep or native or selfplay or device_records or rl" -m gpu -q --timeout 150 --timeout-method thread
step rl 500 python3 -u benchmarks/rl_iteration_benchmark.py --games 20,512 --iterations 2 --records device --drivers native
step vgen 300 python3 -u benchmarks/value_generate_benchmark.py --games 256 --drivers native
