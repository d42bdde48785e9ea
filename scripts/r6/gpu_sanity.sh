#!/bin/bash
# Bench variants after the rows / head changes: graph replay, fp8 precision, torch backend, B = 1 / 4.
O=gpurun_out/r6/sanity
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step graph 300 python bench.py --gpus 1 --steps 20 --warmup 5 --graph
step fp8 300 python bench.py --gpus 1 --steps 20 --warmup 5 --precision fp8
step torch 300 python bench.py --gpus 1 --steps 5 --warmup 2 --backend torch --batch 256
step b1 120 python bench.py --gpus 1 --batch 1 --steps 300 --warmup 50
step b4 120 python bench.py --gpus 1 --batch 4 --steps 300 --warmup 50
step b16g 120 python bench.py --gpus 1 --batch 16 --steps 300 --warmup 50 --graph
for f in $O/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f) $(grep -o '"top1_acc": [0-9.]*' $f)"; done
