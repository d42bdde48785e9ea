#!/bin/bash
# Round 4 batch WG: whole-game self-play to the end on the fp8 engines (256 games, 400 playouts).
O=gpurun_out/r4_wg
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step selfplay 1000 env OUT=$O ALPHAGO_AMD_PRECISION=fp8 GAMES=256 PLAYOUTS=400 MAXMOVES=722 LIMIT=900 PROGRESS=20 bash scripts/selfplay_whole_game.sh
