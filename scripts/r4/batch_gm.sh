#!/bin/bash
# Round 4 batch GM: genmove after the side stream + one-board encode parts; MCTS / search tests.
O=gpurun_out/r4_gm
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_gpu_features.py tests/test_models_play.py tests/test_reference_api.py tests/test_lockstep.py -m gpu -q --timeout 150 --timeout-method thread
step genmove 240 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,16,32 --moves 6
