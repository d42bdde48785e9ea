#!/bin/bash
# fp8 wgrad with carried pixel addressing + MFMA bias / packed amax: tests, kernel probe, value A/B
set -o pipefail
O=gpurun_out/r5/b45
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv160.py tests/test_fp8_inference.py > $O/tests.log 2>&1 &&
P_PROBES=0,2,7,15 timeout -k 10 200 python -u scripts/r5/wgrad_fp8_probe.py > $O/wgrad_probe.log 2>&1 &&
(cd ab_prev && timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8) > $O/value_prev.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8 > $O/value_new.log 2>&1 &&
(cd ab_prev && timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8) > $O/value_prev2.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8 > $O/value_new2.log 2>&1
