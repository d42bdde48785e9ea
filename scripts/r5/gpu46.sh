#!/bin/bash
# bf16 wgrad with carried pixel addressing: wgrad tests + headline bench A/B against the previous tree
set -o pipefail
O=gpurun_out/r5/b46
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_conv160.py -k "wgrad" > $O/tests.log 2>&1 &&
(cd ab_prev && timeout -k 10 400 python -u bench.py --steps 20 --warmup 5) > $O/bench_prev.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_new.log 2>&1 &&
(cd ab_prev && timeout -k 10 400 python -u bench.py --steps 20 --warmup 5) > $O/bench_prev2.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_new2.log 2>&1
