#!/bin/bash
# Round 5, value parity (3 seeds, material task, Adam) + value benchmark quality/speed
set -o pipefail
mkdir -p gpurun_out/r5
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u scripts/value_fp8_parity.py gpurun_out/r5/parity_mat_adam.json --task material \
  --epochs 8 --arms torch-fp32,hip-bf16,hip-fp8,hip-fp8mix,hip-fp8mixsr --optimizer adam --lr 0.0003 --decay 0.001 \
  --seeds 3 > gpurun_out/r5/parity_mat_adam.log 2>&1 || { tail -20 gpurun_out/r5/parity_mat_adam.log; exit 1; }
grep -E "epoch 8|data" gpurun_out/r5/parity_mat_adam.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_distributed_gpu.py -k world4 > gpurun_out/r5/dist4.log 2>&1 || { tail -30 gpurun_out/r5/dist4.log; exit 1; }
tail -2 gpurun_out/r5/dist4.log
for prec in fp8 bf16; do
  timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision $prec --steps 30 \
    > gpurun_out/r5/value_bench_$prec.log 2>&1 || { tail -20 gpurun_out/r5/value_bench_$prec.log; exit 1; }
  tail -1 gpurun_out/r5/value_bench_$prec.log
done
