#!/bin/bash
# Round 4 batch Y: split-K target 144 workgroups (new default) vs 512 (old) -- SL step at B = 1 / 2 / 4
# and graph-timed policy forwards.
O=gpurun_out/r4_y
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 200 python3 -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -k "splitk" -m gpu -q --timeout 150 --timeout-method thread
for W in 144 512; do
  for B in 1 2 4; do
    step sl_b${B}_w$W 120 env ALPHAGO_AMD_SPLITK_WGS=$W python3 bench.py --batch $B --steps 300 --warmup 50 --pool 4096
  done
  step fwd_w$W 120 env ALPHAGO_AMD_SPLITK_WGS=$W python3 benchmarks/forward_latency_benchmark.py --batches 1,2,4
done
