#!/bin/bash
# Round 4 batch R: small-batch forward GPU time (policy / value, bf16 / fp8, B = 1..32).
O=gpurun_out/r4_r
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step fwdlat 300 python3 -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32,64
step fwdlat_nosk 300 env ALPHAGO_AMD_SPLITK=0 python3 -u benchmarks/forward_latency_benchmark.py --batches 1,4
