#!/bin/bash
# Alternating A/B: split-K wgrad reduce on the main stream (0) vs a side stream beside the dgrad (1)
set -e
mkdir -p gpurun_out/rsab
export PYTHONPATH=$PWD
timeout -k 10 120 python -u -m pytest tests/test_determinism_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rsab/tests.log 2>&1
tail -1 gpurun_out/rsab/tests.log
for rep in 1 2 3; do
  for rs in 0 1; do
    timeout -k 10 150 python -u bench.py --steps 40 --warmup 10 --reduce-stream $rs 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('reduce_stream', $rs, d['value'], d['ms_per_step'])" | tee -a gpurun_out/rsab/ab.txt
  done
done
