#!/bin/bash
# SL fp8-forward vs bf16 at the reference learning rate (0.03, supervised_policy_trainer.py -r default),
# 5 seeds, the same task as gpu_b3.sh (which used the round-5 collapse configuration, lr 0.05).
set -o pipefail
O=gpurun_out/r6/fp8lr
mkdir -p $O
export PYTHONUNBUFFERED=1
for s in 0 1 2 3 4; do
  timeout -k 10 240 python scripts/sl_teacher_accuracy.py /tmp/slacc_$s --positions 131072 --epochs 4 --seed $s \
    --lr 0.03 --arms hip-bf16,hip-fp8fwd >> $O/sl_fp8_lr003.jsonl 2> $O/sl_fp8_lr003_$s.err || exit 1
  tail -1 $O/sl_fp8_lr003.jsonl | cut -c1-400
done
