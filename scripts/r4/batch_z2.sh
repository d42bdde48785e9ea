#!/bin/bash
# Round 4 batch Z2: split-K at B = 8 / 16 (ALPHAGO_AMD_SPLITK_MAX_M raised) vs the unsplit 32-pixel tile.
O=gpurun_out/r4_z2
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step fwd_sk 200 env ALPHAGO_AMD_SPLITK_MAX_M=6000 python3 benchmarks/forward_latency_benchmark.py --batches 8,16
step fwd 200 python3 benchmarks/forward_latency_benchmark.py --batches 8,16
for B in 8 16; do
  step sl_b${B}_sk 120 env ALPHAGO_AMD_SPLITK_MAX_M=6000 python3 bench.py --batch $B --steps 300 --warmup 50 --pool 8192
  step sl_b${B} 120 python3 bench.py --batch $B --steps 300 --warmup 50 --pool 8192
done
