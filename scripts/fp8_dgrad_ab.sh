#!/bin/bash
# All-fp8 value backward (fp8 dgrad from the e5m2 copy + fp8 wgrad): numerics, cosine, value-step A/B.
set -e
O=gpurun_out/d8
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 200 python3 -u -m pytest tests/test_conv160.py tests/test_fp8_inference.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 -u scripts/probes/fp8_grad_cosine.py > $O/cosine.jsonl 2>/dev/null
python3 -c "
import json
for l in open('$O/cosine.jsonl'):
    d=json.loads(l); print(d['arm'], d['min_trunk_cos'], d['mean_trunk_cos'])"
for arm in "bf16" "fp8" "fp8 --fp8-dgrad" "bf16" "fp8" "fp8 --fp8-dgrad"; do
  timeout -k 10 180 python3 benchmarks/value_training_benchmark.py --steps 30 --warmup 5 --precision $arm > $O/v.json 2>/dev/null
  echo "$arm: $(python3 -c "import json; d=json.loads(open('$O/v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['mse'])")"
done
