#!/bin/bash
# Round 5 batch 9: split-K at B = 16..64 (SPLITK_MAX_M raised) and its workgroup target: forward latency + SL step
O=gpurun_out/r5/b9
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
source scripts/r5/lib.sh
step fwd_base 300 python -u benchmarks/forward_latency_benchmark.py --batches 8,16,32,64 --iters 30
for w in 256 384 512 768; do
  step fwd_sk$w 300 env ALPHAGO_AMD_SPLITK_MAX_M=40000 ALPHAGO_AMD_SPLITK_WGS=$w python -u benchmarks/forward_latency_benchmark.py --batches 8,16,32,64 --iters 30
done
for w in 0 384 512; do
  if [ $w = 0 ]; then E=""; else E="ALPHAGO_AMD_SPLITK_MAX_M=40000 ALPHAGO_AMD_SPLITK_WGS=$w"; fi
  step sl16_sk$w 300 env $E python -u bench.py --batch 16 --steps 200 --warmup 20 --pool 4096
  step sl32_sk$w 300 env $E python -u bench.py --batch 32 --steps 200 --warmup 20 --pool 4096
done
grep -h '"batch"' $O/fwd_*.log | grep policy | grep bf16 > $O/fwd_policy_bf16.txt || true
