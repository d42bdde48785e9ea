#!/bin/bash
# Alternating A/B of the SL bench: the session-start tree (ab_old/, python from 78f57de with the
# current .so files) vs HEAD, to separate box-to-box variance from a code regression.
set -e
mkdir -p gpurun_out/abold
for rep in 1 2 3; do
  (cd ab_old && PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 40 --warmup 5 2>/dev/null) | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('old', d['value'], d['ms_per_step'])" | tee -a gpurun_out/abold/ab.txt
  PYTHONPATH=$PWD timeout -k 10 200 python bench.py --steps 40 --warmup 5 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('head', d['value'], d['ms_per_step'])" | tee -a gpurun_out/abold/ab.txt
done
