#!/bin/bash
# Round-6 batch 5: RL learning-rate sweep against the fixed SL net (pool = the SL net only), each RL net
# then matched against SL over 1000 games; split-free wgrad at ksub 1 / 2 / 4.
O=gpurun_out/r6/ev
mkdir -p $O gpurun_out/r6/b5
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
O2=$O
for lr in 0.003 0.01; do
  O=$O2 step rl_lr$lr 300 python scripts/r6/evidence.py rl $O2 --nets r6_nets --tag _lr$lr --games 512 \
    --iterations 40 --save-every 40 --lr $lr --batch 1024
  O=$O2 step match_lr$lr 120 python scripts/r6/evidence.py match $O2 --nets r6_nets --tag _lr$lr --games 1000
  mkdir -p gpurun_out/r6/nets && cp r6_nets/rl_lr$lr.* gpurun_out/r6/nets/
done
O=gpurun_out/r6/b5
step wgrad_direct_bench 300 python scripts/r6/wgrad_direct_bench.py
step direct_tests 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "wgrad_direct"
cat gpurun_out/r6/b5/wgrad_direct_bench.log
for f in $O2/match_rl_lr*_vs_sl.json; do echo $f; grep -E "rl_win_rate|ci95" -A2 $f | head -5; done
