#!/bin/bash
# Round 5 batch 5: GPU suite (deferred reduce + retirement), bench A/B of the deferred reduce, in-step trace
O=gpurun_out/r5/b5
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
source scripts/r5/lib.sh
SECONDS=0
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo "suite wall ${SECONDS} s"
grep -E "passed|failed" $O/suite.log | tail -2
for r in 1 2; do
  for d in 1 0; do
    ALPHAGO_AMD_DEFER_REDUCE=$d step bench_defer${d}_$r 300 python -u bench.py --steps 40 --warmup 5
  done
done
prof trace_b2176 300 10 --steps 10 --warmup 5 --min-warmup-s 0
