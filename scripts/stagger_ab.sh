#!/bin/bash
# Wave-group stagger (tile 388) vs tile 386: conv numerics, then alternating same-box benches.
set -e
O=gpurun_out/stg
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_conv160.py -m gpu -x -q -k "388" \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for t in 386 388; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --conv-tile $t > $O/sl_$t.json 2>/dev/null
    echo "$r SL tile $t $(python3 -c "import json; d=json.loads(open('$O/sl_$t.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
for t in 386 388; do
  timeout -k 10 200 python3 benchmarks/value_training_benchmark.py --precision bf16 --conv-tile $t > $O/v_$t.json 2>/dev/null
  echo "value bf16 tile $t $(python3 -c "import json; d=json.loads(open('$O/v_$t.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
