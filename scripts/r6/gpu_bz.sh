#!/bin/bash
# Round-6 batch Z: search vs the greedy raw policy with per-pair random openings (the first run had two
# distinct games: both players deterministic); RL with the opponent pool and the mean-outcome baseline.
O=gpurun_out/r6/ev
mkdir -p $O gpurun_out/r6/nets
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step search2 760 python scripts/r6/evidence.py search $O --nets r6_nets --games 200 --playouts 1600 --leaves 32 \
  --opening 8 --latency-moves 40
step rl_poolb 420 python scripts/r6/evidence.py rl $O --nets r6_nets --tag _poolb_lr0.01 --games 512 \
  --iterations 100 --save-every 10 --lr 0.01 --batch 1024
step match_poolb 120 python scripts/r6/evidence.py match $O --nets r6_nets --tag _poolb_lr0.01 --games 1000
cp r6_nets/rl_poolb_lr0.01.* gpurun_out/r6/nets/ 2>/dev/null
grep -E "mcts_win_rate|ci95|genmove" -A2 $O/search_vs_policy.json | head -12
grep -E "rl_win_rate|ci95" -A2 $O/match_rl_poolb_lr0.01_vs_sl.json | head -5
