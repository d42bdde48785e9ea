#!/bin/bash
# Round 4 batch U: fp8 engine threshold (tests; forward GPU time with the fp8 trunk forced at every batch
# to place the bf16 / fp8 crossover).  Output: gpurun_out/r4_u/
O=gpurun_out/r4_u
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_fp8_inference.py -m gpu -q --timeout 150 --timeout-method thread
step fwdlat_fp8all 300 env ALPHAGO_AMD_FP8_MIN_BATCH=0 python3 -u benchmarks/forward_latency_benchmark.py --batches 64,128,256,512,1024 --iters 30
step fwdlat_default 300 python3 -u benchmarks/forward_latency_benchmark.py --batches 1,16,64,128,256 --iters 30
