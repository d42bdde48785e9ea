#!/bin/bash
# fp8 value-training check: fp8 conv tests, wgrad kernel A/B, gradient cosine
# vs bf16, and the value-training benchmark in each precision arm.  Output: gpurun_out/fp8v/
set -e
O=gpurun_out/fp8v
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_conv160.py tests/test_fp8_inference.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 -u scripts/probes/wgrad_fp8_bench.py 1024 3 > $O/wgrad_ab.jsonl 2>&1
cat $O/wgrad_ab.jsonl
timeout -k 10 120 python3 -u scripts/probes/fp8_grad_cosine.py > $O/cosine.jsonl 2>&1
cut -c1-200 $O/cosine.jsonl
for arm in "bf16" "fp8" "fp8 --fp8-wgrad" "fp8 --fp8-dgrad --fp8-wgrad"; do
    timeout -k 10 180 python3 benchmarks/value_training_benchmark.py --steps 30 --warmup 5 --precision $arm \
        >> $O/value.jsonl 2>> $O/value.err
    tail -1 $O/value.jsonl | cut -c1-200
done
