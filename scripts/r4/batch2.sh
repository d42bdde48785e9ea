#!/bin/bash
# Round 4 batch: lock-step driver tests + throughput, small-batch kernels (numerics, timings, SL step),
# packed-tap first layer, value fp8 parity.  Output: gpurun_out/r4_b2/
O=gpurun_out/r4_b2
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step kernels 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_conv160.py tests/test_hip_trainer.py tests/test_fp8_inference.py -x -q --timeout 120 --timeout-method thread
step lockstep_tests 300 python3 -u -m pytest tests/test_lockstep.py tests/test_rl_value.py -m gpu -x -v --timeout 150 --timeout-method thread
step kbench 200 python3 -u scripts/r4/small_batch_kbench.py 1 4 16 64 256
cp $O/kbench.log $O/kbench.jsonl
step bench2176 240 python3 bench.py --gpus 1 --steps 20 --warmup 5
for B in 16 64 256; do
  for T in 0 65; do
    step sl_b${B}_t${T} 120 python3 bench.py --batch $B --steps 200 --warmup 50 --conv-tile $T --pool 8192
  done
done
step rl 500 python3 -u benchmarks/rl_iteration_benchmark.py --games 20,512 --iterations 1 --records device
step vgen 400 python3 -u benchmarks/value_generate_benchmark.py --games 256
step value_parity 600 python3 -u scripts/value_fp8_parity.py $O/value_parity.json --positions 32768 --epochs 4
step genmove 300 python3 -u benchmarks/genmove_benchmark.py --playouts 1600 --leaves 8,16,32 --moves 4
step value_fp8 200 python3 -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30 --warmup 10
step value_bf16 200 python3 -u benchmarks/value_training_benchmark.py --precision bf16 --steps 30 --warmup 10
step prof 300 bash scripts/profile_step.sh $O/prof --steps 20 --warmup 5
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1; cat $O/timeline.txt | head -30
