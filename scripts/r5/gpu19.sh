#!/bin/bash
# weight-stationary with the LDS input-row ring: tests, per-layer times, probes
O=gpurun_out/r5/b19
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step ws_test 300 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -x -q --timeout 120 --timeout-method thread -k "weight_stationary or splitk"
grep -E "passed|failed" $O/ws_test.log | tail -2
grep -q " passed" $O/ws_test.log && ! grep -q "failed" $O/ws_test.log || exit 1
step ws_bench 300 env WS_BATCHES=1,4,8,16,32,64 python -u scripts/r5/ws_bench.py
grep '"C"' $O/ws_bench.log
step probes 300 env WS_WIDTHS=192 WS_BATCHES=1,8,16 WS_TILES=40,1002,1004,1008,1014 python -u scripts/r5/ws_bench.py
grep '"C"' $O/probes.log
