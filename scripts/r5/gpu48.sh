#!/bin/bash
# fp8 wgrad with LDS-direct buffer loads (32-bit offsets): wgrad tests, kernel time, value bench
set -o pipefail
O=gpurun_out/r5/b48
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv160.py tests/test_fp8_inference.py > $O/tests.log 2>&1 &&
P_PROBES=0 timeout -k 10 200 python -u scripts/r5/wgrad_fp8_probe.py > $O/wgrad.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8 > $O/value_fp8.log 2>&1 &&
P_PROBES=0 timeout -k 10 200 python -u scripts/r5/wgrad_fp8_probe.py > $O/wgrad2.log 2>&1
