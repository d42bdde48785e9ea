#!/bin/bash
# SL fp8-forward: round-to-nearest vs stochastic rounding over seeds 1 / 2 (4 epochs, lr 0.05)
O=gpurun_out/r5/b37
mkdir -p $O /tmp/slacc
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
for s in 1 2; do
  step rn$s 600 python -u scripts/sl_teacher_accuracy.py /tmp/slacc/rn$s --positions 131072 --epochs 4 --arms hip-fp8fwd,hip-bf16 --seed $s
  tail -1 $O/rn$s.log | cut -c1-700
  step sr$s 600 env ALPHAGO_AMD_FP8_SR=1 python -u scripts/sl_teacher_accuracy.py /tmp/slacc/sr$s --positions 131072 --epochs 4 --arms hip-fp8fwd --seed $s
  tail -1 $O/sr$s.log | cut -c1-400
done
