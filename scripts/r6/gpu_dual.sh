#!/bin/bash
# Round-6: dual-split wgrad (two pixel splits per 1024-thread workgroup, half the slab) -- numerics,
# then the headline A/B (alternating, same box) and its step timeline.
O=gpurun_out/r6/dual
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step dual_test 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "wgrad_dual or test_conv_wgrad"
for rep in 1 2 3; do
  for d in 0 1; do
    step head_d${d}_r$rep 150 python bench.py --wgrad-dual $d --steps 30 --warmup 10
  done
done
prof prof_dual 300 5 --wgrad-dual 1 --steps 10 --warmup 5
grep -h '"value"' $O/head_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'].get('wgrad_dual'), d['value'], d['ms_per_step'])
"
