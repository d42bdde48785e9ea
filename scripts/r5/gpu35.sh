#!/bin/bash
# final numbers: value benchmark (speed + 1600-step quality), genmove, forward latency
O=gpurun_out/r5/b35
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step value_fp8 600 python -u benchmarks/value_training_benchmark.py --precision fp8
grep -h '^{' $O/value_fp8.log | cut -c1-700
step value_bf16 600 python -u benchmarks/value_training_benchmark.py --precision bf16
grep -h '^{' $O/value_bf16.log | cut -c1-700
step gm_pos 600 python -u benchmarks/genmove_benchmark.py --positions benchmarks/data/lee_sedol_positions.json --leaves 32
step gm_empty 600 python -u benchmarks/genmove_benchmark.py --leaves 16,32 --moves 10
grep -h ms_ $O/gm_*.log | cut -c1-300
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32,64 --iters 30
grep bf16 $O/fwd_lat.log
