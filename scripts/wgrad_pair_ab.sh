#!/bin/bash
# Tap-pair wgrad (variant 6) vs the per-tap kernel: numerics, 10 s power-limited A/B, bench A/B.
set -e
O=gpurun_out/wpair
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py -m gpu -x -q -k "wgrad" \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
OUT=$O KERNELS="wgrad:0 wgrad:6 wgrad:8 wgrad:0 wgrad:6 wgrad:8" SECS=${SECS:-8} bash scripts/conv_power_ab.sh > /dev/null 2>&1
cat $O/result.txt
for v in 0 6 8; do
  ALPHAGO_AMD_WGRAD_VARIANT=$v timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err
  echo "variant $v: $(python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
