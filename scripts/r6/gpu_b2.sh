#!/bin/bash
# Round-6 batch 2: evidence stage 1 (SL -> RL -> match), then the split-free wgrad tests + microbench.
set -o pipefail
O=gpurun_out/r6/ev
mkdir -p $O gpurun_out/r6/b2
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/r6/evidence.py sl $O --positions 262144 --epochs 6 --batch 256 --lr 0.05 > $O/sl.log 2>&1 &&
timeout -k 10 600 python scripts/r6/evidence.py rl $O --games 512 --iterations 100 --save-every 10 --lr 0.03 --batch 1024 > $O/rl.log 2>&1 &&
timeout -k 10 240 python scripts/r6/evidence.py match $O --games 1000 > $O/match.log 2>&1
rc=$?
tail -3 $O/*.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "wgrad_direct or weight_stationary or test_conv_wgrad" > gpurun_out/r6/b2/tests.log 2>&1 &&
timeout -k 10 300 python scripts/r6/wgrad_direct_bench.py > gpurun_out/r6/b2/wgrad_direct_bench.jsonl 2> gpurun_out/r6/b2/wgrad_direct_bench.err
rc=$?
tail -5 gpurun_out/r6/b2/tests.log; cat gpurun_out/r6/b2/wgrad_direct_bench.jsonl
exit $rc
