#!/bin/bash
# Round 4 batch K: split-K small-batch conv (tests, SL B = 16 / 4 A/B, B = 16 trace, genmove), then a
# learnability sweep of the value parity task (hip-bf16 arm only).  Output: gpurun_out/r4_k/
O=gpurun_out/r4_k
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -k "splitk or small_batch or thin_input or packed_tap or fused_sgd" -m gpu -q --timeout 150 --timeout-method thread
step sl16_sk 120 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192
step sl16_nosk 120 env ALPHAGO_AMD_SPLITK=0 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192
step sl16_sk2 120 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192
step sl4_sk 120 python3 bench.py --batch 4 --steps 300 --warmup 50 --pool 4096
step sl4_nosk 120 env ALPHAGO_AMD_SPLITK=0 python3 bench.py --batch 4 --steps 300 --warmup 50 --pool 4096
step sl64_sk 120 python3 bench.py --batch 64 --steps 300 --warmup 50 --pool 8192
prof prof16 200 200 --batch 16 --steps 200 --warmup 50 --pool 8192
step genmove 240 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,32 --moves 4
for init in keras he; do
  for lr in 0.005 0.02 0.05; do
    step sweep_material_${init}_${lr} 120 python3 -u scripts/value_fp8_parity.py $O/sweep_material_${init}_${lr}.json --task material --init $init --lr $lr --positions 16384 --heldout 4096 --epochs 8 --arms hip-bf16
  done
done
step sweep_teacher_he_0.02 120 python3 -u scripts/value_fp8_parity.py $O/sweep_teacher_he_0.02.json --task teacher --init he --lr 0.02 --positions 16384 --heldout 4096 --epochs 8 --arms hip-bf16
