#!/bin/bash
set -e
O=gpurun_out/gs
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_determinism_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 benchmarks/graph_step_benchmark.py --batches 16,64,256 > $O/graph_step.jsonl 2>/dev/null
cat $O/graph_step.jsonl
