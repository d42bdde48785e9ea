#!/bin/bash
# Round 4: the ADVICE regression tests (fp8 wgrad exponents, fp8 overlap join, device records),
# a driver-shaped bench and the real-move (Lee Sedol held-out game) accuracy check.
# Output: gpurun_out/r4_advice/
set -e
O=gpurun_out/r4_advice
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err
tail -1 $O/bench1.json | cut -c1-260
timeout -k 10 400 python3 -u -m pytest tests/test_fp8_inference.py tests/test_rl_value.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
timeout -k 10 500 python3 -u scripts/sl_teacher_accuracy.py /tmp/r4_real --real-only --real-epochs 40 --real-seeds 5 \
  --real-lr 0.03 --arms hip-bf16,torch-fp32 > $O/real_moves.json 2> $O/real_moves.err
tail -1 $O/real_moves.json
