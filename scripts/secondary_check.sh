#!/bin/bash
# Secondary benchmarks at the current head (each step under its own time limit, stop at the first failure)
set -e
O=gpurun_out/sec
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python benchmarks/selfplay_dp_benchmark.py --playouts 1600 --moves 2 > $O/selfplay_bf16.log 2>&1
tail -1 $O/selfplay_bf16.log | cut -c1-400
ALPHAGO_AMD_PRECISION=fp8 timeout -k 10 300 python benchmarks/selfplay_dp_benchmark.py --playouts 1600 --moves 2 > $O/selfplay_fp8.log 2>&1
tail -1 $O/selfplay_fp8.log | cut -c1-400
timeout -k 10 300 python benchmarks/value_training_benchmark.py --precision bf16 > $O/value_bf16.log 2>&1
tail -1 $O/value_bf16.log | cut -c1-400
timeout -k 10 300 python benchmarks/value_training_benchmark.py --precision fp8 > $O/value_fp8.log 2>&1
tail -1 $O/value_fp8.log | cut -c1-400
timeout -k 10 300 python benchmarks/inference_benchmark.py > $O/inference.log 2>&1
tail -3 $O/inference.log | cut -c1-400
