#!/bin/bash
# Round 4 batch Q: fp8 tests + value fp8 step after the weight-scale pass change; whole-game batched MCTS
# self-play with a 722-move cap (games end by two passes / resignation; endings counted in the summary).
# Output: gpurun_out/r4_q/
O=gpurun_out/r4_q
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step fp8tests 300 python3 -u -m pytest tests/test_fp8_inference.py tests/test_conv160.py -m gpu -q --timeout 150 --timeout-method thread
step value_fp8 240 python3 -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30 --warmup 10
step selfplay 1000 env OUT=$O GAMES=256 PLAYOUTS=400 MAXMOVES=722 LIMIT=900 PROGRESS=20 bash scripts/selfplay_whole_game.sh
