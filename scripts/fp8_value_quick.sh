#!/bin/bash
# fp8 value path: GPU tests of the fp8 kernels, then the value benchmark (bf16 / all-fp8), kernel stats.
set -e
O=gpurun_out/fq
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 200 python3 -u -m pytest tests/test_conv160.py tests/test_fp8_inference.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for arm in "bf16" "fp8" "bf16" "fp8"; do
  timeout -k 10 180 python3 benchmarks/value_training_benchmark.py --steps 30 --warmup 5 --precision $arm > $O/v.json 2>/dev/null
  echo "$arm: $(python3 -c "import json; d=json.loads(open('$O/v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 benchmarks/value_training_benchmark.py --steps 20 --warmup 5 > $O/prof.log 2>&1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/value_kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/value_kernel_stats.csv')))[:12]: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Percentage'])"
