#!/bin/bash
# Round-6 batch V: RL with the opponent pool, baseline, gradient clip 5, weight decay 1e-4, evaluation vs
# SL every 5 iterations (200 games) keeping the best snapshot; fresh 1000-game matches of the kept nets.
O=gpurun_out/r6/ev
mkdir -p $O gpurun_out/r6/nets
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
for lr in 0.01 0.003; do
  step rl_sel_lr$lr 480 python scripts/r6/evidence.py rl $O --nets r6_nets --tag _sel_lr$lr --games 512 \
    --iterations 100 --save-every 10 --lr $lr --batch 1024 --clip 5 --wd 1e-4 --eval-every 5 --seed 1
  step match_sel_lr$lr 120 python scripts/r6/evidence.py match $O --nets r6_nets --tag _sel_lr$lr --games 1000 --seed 5
  grep -E "rl_win_rate|ci95" -A2 $O/match_rl_sel_lr${lr}_vs_sl.json | head -5
done
cp r6_nets/rl_sel_lr*.* gpurun_out/r6/nets/ 2>/dev/null
