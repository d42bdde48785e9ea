#!/bin/bash
# fp8 160-wide forward/dgrad with 4-wave workgroups + staged byte outputs: tests, kernel A/B against
# the round-4 tiling (lab 6), value fp8 training A/B against the previous tree (ab_prev, same box)
set -o pipefail
O=gpurun_out/r5/b42
mkdir -p $O
export ALPHAGO_AMD_LAB_TESTS=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv160.py tests/test_fp8_inference.py > $O/tests.log 2>&1 &&
P_VARIANTS=0,6 P_OUT=fp8mb timeout -k 10 200 python -u scripts/r5/fp8_probe2.py > $O/fwd_fp8mb.log 2>&1 &&
P_VARIANTS=0,6 timeout -k 10 200 python -u scripts/r5/fp8_probe2.py > $O/fwd_both.log 2>&1 &&
(cd ab_prev && timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8) > $O/value_prev.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8 > $O/value_new.log 2>&1 &&
(cd ab_prev && timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8) > $O/value_prev2.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/value_training_benchmark.py --precision fp8 > $O/value_new2.log 2>&1
