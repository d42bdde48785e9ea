#!/bin/bash
# Round-6 batch W: RL with the opponent pool, the mean-outcome baseline and gradient-norm clipping
# (100 x 512 games; lr 0.01 and 0.003), each matched against SL over 1000 games.
O=gpurun_out/r6/ev
mkdir -p $O gpurun_out/r6/nets
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
for lr in 0.01 0.003; do
  step rl_final_lr$lr 420 python scripts/r6/evidence.py rl $O --nets r6_nets --tag _final_lr$lr --games 512 \
    --iterations 100 --save-every 10 --lr $lr --batch 1024 --clip 5
  step match_final_lr$lr 120 python scripts/r6/evidence.py match $O --nets r6_nets --tag _final_lr$lr --games 1000
  grep -E "rl_win_rate|ci95" -A2 $O/match_rl_final_lr${lr}_vs_sl.json | head -5
done
cp r6_nets/rl_final_lr*.* gpurun_out/r6/nets/ 2>/dev/null
