#!/bin/bash
# Round 4 batch F: value training speed + held-out MSE on the value-teacher task (fp8 / bf16),
# real-move accuracy (Lee Sedol held-out game), single-tree genmove latency.  Output: gpurun_out/r4_f/
O=gpurun_out/r4_f
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
# step fp8tests 300 python3 -u -m pytest tests/test_fp8_inference.py -m gpu -q -s --timeout 150 --timeout-method thread
step value_fp8 240 python3 -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30 --warmup 10
step value_bf16 240 python3 -u benchmarks/value_training_benchmark.py --precision bf16 --steps 30 --warmup 10
step real_moves 420 python3 -u scripts/sl_teacher_accuracy.py /tmp/r4_real --real-only --real-epochs 40 --real-seeds 5 --real-lr 0.03 --arms hip-bf16,torch-fp32
step genmove 240 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,16,32 --moves 4
