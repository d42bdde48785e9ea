#!/bin/bash
# Round 5 batch 7: GPU suite (retirement, half-width layer-0 wgrad default), tail-overlap A/B + trace
O=gpurun_out/r5/b7
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
source scripts/r5/lib.sh
SECONDS=0
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo "suite wall ${SECONDS} s"
for r in 1 2; do
  for t in 1 0; do
    step bench_tail${t}_$r 300 env ALPHAGO_AMD_TAIL_OVERLAP=$t python -u bench.py --steps 40 --warmup 5
  done
done
ALPHAGO_AMD_TAIL_OVERLAP=1 prof trace_tail1 300 10 --steps 10 --warmup 5 --min-warmup-s 0
