#!/bin/bash
# Round 5 batch 8: value benchmark (material task, train-value defaults), 5-seed value parity
O=gpurun_out/r5/b8
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
source scripts/r5/lib.sh
for prec in fp8 bf16; do
  step value_bench_$prec 300 python -u benchmarks/value_training_benchmark.py --precision $prec --steps 30
done
step parity5 1000 python -u scripts/value_fp8_parity.py $O/parity_mat_adam5.json --task material \
  --epochs 8 --arms torch-fp32,hip-bf16,hip-fp8,hip-fp8mix --optimizer adam --lr 0.0003 --decay 0.005 --seeds 5
grep "epoch 8" $O/parity5.log
