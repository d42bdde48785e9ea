#!/bin/bash
# Round 4 batch SP: the round-3 self-play configuration (fp8 engines, 256 games, 1600 playouts) over the
# first 100 moves, for a same-configuration comparison with profiles/r3_selfplay (258.0k / 248.9k leaf
# evaluations/s in moves 0-49 / 50-99).
O=gpurun_out/r4_sp
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step selfplay 600 env OUT=$O ALPHAGO_AMD_PRECISION=fp8 GAMES=256 PLAYOUTS=1600 MAXMOVES=100 LIMIT=560 PROGRESS=10 bash scripts/selfplay_whole_game.sh
