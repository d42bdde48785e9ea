#!/bin/bash
# Round 4 native lock-step driver: equality tests vs the Python loop, RL iteration and value-generate
# throughput (native vs python).  Output: gpurun_out/r4_lockstep/
set -e
O=gpurun_out/r4_lockstep
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_lockstep.py tests/test_rl_value.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python3 -u benchmarks/rl_iteration_benchmark.py --games 20,512 --iterations 1 --records device > $O/rl.jsonl 2> $O/rl.err
cat $O/rl.jsonl
timeout -k 10 300 python3 -u benchmarks/value_generate_benchmark.py --games 256 > $O/vgen.jsonl 2> $O/vgen.err
cat $O/vgen.jsonl
