#!/bin/bash
# Round 5, first GPU pass: new optimizer / fallback tests, value-learning sweep on the material task, bench.
set -o pipefail
mkdir -p gpurun_out/r5
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_hip_trainer.py tests/test_gpu_features.py -k "optimizer or overflow or two_batches or fused_sgd" \
  > gpurun_out/r5/tests1.log 2>&1 || { tail -30 gpurun_out/r5/tests1.log; exit 1; }
tail -3 gpurun_out/r5/tests1.log
for cfg in "adam 0.0003 keras" "adam 0.0001 he" "momentum 0.003 he"; do
  set -- $cfg
  timeout -k 10 420 python -u scripts/value_fp8_parity.py gpurun_out/r5/mat_$1_$2_$3.json --task material \
    --epochs 8 --arms torch-fp32,hip-bf16 --optimizer $1 --lr $2 --init $3 > gpurun_out/r5/mat_$1_$2_$3.log 2>&1 \
    || { tail -20 gpurun_out/r5/mat_$1_$2_$3.log; exit 1; }
  grep -E "epoch 8|data" gpurun_out/r5/mat_$1_$2_$3.log
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench1.log 2>&1 || { tail -20 gpurun_out/r5/bench1.log; exit 1; }
tail -1 gpurun_out/r5/bench1.log
