#!/bin/bash
# staged byte outputs on the 192-wide fp8 tile: fp8 tests (lab equality included), inference bench
set -o pipefail
O=gpurun_out/r5/b50
mkdir -p $O
ALPHAGO_AMD_LAB_TESTS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv160.py tests/test_fp8_inference.py > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k fp8 > $O/tests_hk.log 2>&1
