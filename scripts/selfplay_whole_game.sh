#!/bin/bash
# Whole-game batched MCTS self-play throughput: GAMES concurrent games (one tree each) x PLAYOUTS
# simulations per move, policy 12x192 + value 12x152 (random init), played to the end (two passes,
# resignation or MAXMOVES).  Records go to /tmp (large); the summary with the per-phase table to OUT.
set -e
OUT=${OUT:-gpurun_out/selfplay}
W=${WORK:-/tmp/sp_work}
mkdir -p "$OUT" "$W"
export PYTHONPATH=$PWD
python -m alphago_amd init-model policy "$W/pol.json" --weights "$W/pol.h5" --filters 192 --seed 1 > /dev/null
python -m alphago_amd init-model value "$W/val.json" --weights "$W/val.h5" --filters 152 --seed 2 > /dev/null
timeout -k 10 ${LIMIT:-1000} python -u -m alphago_amd selfplay-mcts "$W/pol.json" "$W/run" --value-json "$W/val.json" \
  --games ${GAMES:-256} --concurrent ${GAMES:-256} --playouts ${PLAYOUTS:-1600} --max-moves ${MAXMOVES:-722} \
  --progress-every ${PROGRESS:-10} --positions-per-game ${PPG:-4} ${EXTRA:-} | tee "$OUT/selfplay.log"
cp "$W/run/selfplay_summary.json" "$OUT/"
ls "$W/run/sgf/rank0" | head -3 > "$OUT/sgf_files.txt"
cp "$W/run/sgf/rank0/game_000000.sgf" "$OUT/" 2>/dev/null || true
