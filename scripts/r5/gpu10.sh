#!/bin/bash
O=gpurun_out/r5/b10
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1
source scripts/r5/lib.sh
step ws_test 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k weight_stationary
grep -E "PASS|FAIL|Error" $O/ws_test.log | head -20
step ws_bench 300 python -u scripts/r5/ws_bench.py
cat $O/ws_bench.log
