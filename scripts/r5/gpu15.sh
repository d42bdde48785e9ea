#!/bin/bash
# WS v2 + ladder cache: full GPU suite, genmove on the Lee Sedol positions (cache on / off), SL sweep
O=gpurun_out/r5/b15
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -E "passed|failed" $O/suite.log | tail -2
step gm_cache 600 python -u benchmarks/genmove_benchmark.py --positions benchmarks/data/lee_sedol_positions.json --leaves 32 --ladder-cache 1
step gm_nocache 600 python -u benchmarks/genmove_benchmark.py --positions benchmarks/data/lee_sedol_positions.json --leaves 32 --ladder-cache 0
for B in 1 4 8 16; do
  step sl$B 300 python -u bench.py --batch $B --steps 200 --warmup 20
done
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32 --iters 30
grep bf16 $O/fwd_lat.log
