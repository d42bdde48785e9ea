#!/bin/bash
# Round 4 batch O: fp8 stochastic rounding (test + value parity arm), the full GPU suite after the
# round-4 changes, smoke, a driver-shaped bench.  Output: gpurun_out/r4_o/
O=gpurun_out/r4_o
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step srtest 200 python3 -u -m pytest tests/test_fp8_inference.py -k "stochastic or fp8_value_training or fp8_backward" -m gpu -q --timeout 150 --timeout-method thread
step value_parity 900 python3 -u scripts/value_fp8_parity.py $O/value_parity.json --task teacher --init he --lr 0.01 --positions 32768 --heldout 8192 --epochs 16 --arms hip-bf16,hip-fp8,hip-fp8sr
step suite 600 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider --durations=10
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 240 python3 bench.py --gpus 1 --steps 20 --warmup 5
