#!/bin/bash
# Round 5: full GPU suite after the lab retirement (wall time), value benchmark, 5-seed value parity
set -o pipefail
mkdir -p gpurun_out/r5
export PYTHONUNBUFFERED=1
SECONDS=0; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5/gpu_suite.log 2>&1 || { tail -40 gpurun_out/r5/gpu_suite.log; exit 1; }
tail -3 gpurun_out/r5/gpu_suite.log; echo "suite wall ${SECONDS} s"
for prec in fp8 bf16; do
  timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision $prec --steps 30 \
    > gpurun_out/r5/value_bench_$prec.log 2>&1 || { tail -20 gpurun_out/r5/value_bench_$prec.log; exit 1; }
  tail -1 gpurun_out/r5/value_bench_$prec.log
done
timeout -k 10 900 python -u scripts/value_fp8_parity.py gpurun_out/r5/parity_mat_adam5.json --task material \
  --epochs 8 --arms torch-fp32,hip-bf16,hip-fp8,hip-fp8mix --optimizer adam --lr 0.0003 --decay 0.005 \
  --seeds 5 > gpurun_out/r5/parity_mat_adam5.log 2>&1 || { tail -20 gpurun_out/r5/parity_mat_adam5.log; exit 1; }
grep -E "epoch 8" gpurun_out/r5/parity_mat_adam5.log
