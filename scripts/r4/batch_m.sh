#!/bin/bash
# Round 4 batch M: learnability sweep 2 for the value parity run (hip-bf16 arm), split-K at B <= 9,
# the full GPU suite with its wall time.  Output: gpurun_out/r4_m/
O=gpurun_out/r4_m
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
for lr in 0.005 0.01; do
  step sweep_teacher_he_$lr 150 python3 -u scripts/value_fp8_parity.py $O/sweep_teacher_he_$lr.json --task teacher --init he --lr $lr --positions 32768 --heldout 8192 --epochs 16 --arms hip-bf16
done
for lr in 0.05 0.1; do
  step sweep_material_keras_$lr 150 python3 -u scripts/value_fp8_parity.py $O/sweep_material_keras_$lr.json --task material --init keras --lr $lr --positions 32768 --heldout 8192 --epochs 16 --arms hip-bf16
done
step sl8_sk 120 python3 bench.py --batch 8 --steps 300 --warmup 50 --pool 4096
step sl8_nosk 120 env ALPHAGO_AMD_SPLITK=0 python3 bench.py --batch 8 --steps 300 --warmup 50 --pool 4096
step sl1_sk 120 python3 bench.py --batch 1 --steps 300 --warmup 50 --pool 1024
step sl1_nosk 120 env ALPHAGO_AMD_SPLITK=0 python3 bench.py --batch 1 --steps 300 --warmup 50 --pool 1024
step genmove 240 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,32 --moves 4
step suite 900 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider --durations=15
