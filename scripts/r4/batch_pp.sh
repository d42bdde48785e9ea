#!/bin/bash
# Round 4 batch PP: single-tree search with two leaf batches in flight -- tests, genmove on / off.
O=gpurun_out/r4_pp${PPTAG:-}
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_gpu_features.py tests/test_models_play.py tests/test_reference_api.py -k "mcts or MCTS or search or play or gtp" -m gpu -q --timeout 150 --timeout-method thread
step gen_on 240 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,16,32 --moves 6
step gen_off 240 env ALPHAGO_AMD_MCTS_PIPELINE=0 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,16,32 --moves 6
