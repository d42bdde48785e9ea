#!/bin/bash
# Round-6 batch 8: RL with the opponent pool (lr 0.01, 100 x 512 games, a snapshot every 10 iterations)
# + 1000-game match vs SL; then the small-batch SL sweep (batch 4).
O=gpurun_out/r6/ev
mkdir -p $O gpurun_out/r6/nets
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step rl_pool 420 python scripts/r6/evidence.py rl $O --nets r6_nets --tag _pool_lr0.01 --games 512 \
  --iterations 100 --save-every 10 --lr 0.01 --batch 1024
step match_pool 120 python scripts/r6/evidence.py match $O --nets r6_nets --tag _pool_lr0.01 --games 1000
cp r6_nets/rl_pool_lr0.01.* gpurun_out/r6/nets/ 2>/dev/null
grep -E "rl_win_rate|ci95" -A2 $O/match_rl_pool_lr0.01_vs_sl.json | head -5
bash scripts/r6/gpu_b4.sh
