#!/bin/bash
# fp8 wgrad: block vs line staging (AGK_WGRAD_FP8_LINE), numerics + kernel A/B + value-step A/B.
set -e
O=gpurun_out/w8
mkdir -p $O
export PYTHONPATH=$PWD
for L in 1 0; do
  AGK_WGRAD_FP8_LINE=$L timeout -k 10 200 python3 -u -m pytest tests/test_conv160.py tests/test_fp8_inference.py -m gpu -x -q \
      --timeout 120 --timeout-method thread > $O/tests_$L.log 2>&1 || { tail -30 $O/tests_$L.log; exit 1; }
  echo "line=$L $(tail -1 $O/tests_$L.log)"
done
for L in 1 0 1; do
  AGK_WGRAD_FP8_LINE=$L timeout -k 10 60 python3 -u scripts/probes/wgrad_fp8_bench.py 1024 2 2>/dev/null | grep fp8 | tail -1 | sed "s/^/line=$L /"
done
for arm in "bf16" "fp8" "fp8 --fp8-wgrad"; do
  timeout -k 10 180 python3 benchmarks/value_training_benchmark.py --steps 30 --warmup 5 --precision $arm > $O/v.json 2>/dev/null
  echo "$arm: $(python3 -c "import json; d=json.loads(open('$O/v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
