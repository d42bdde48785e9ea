#!/bin/bash
# Minibatch gather fused into the input pack (rows) + the value head's column sums on head_grad_sums:
# tests, the driver's bench command, value training, both step timelines.
O=gpurun_out/r6/rows
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step tests 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py tests/test_rl_value.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step value_fp8 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
step value_bf16 300 python -u benchmarks/value_training_benchmark.py --precision bf16 --steps 30
prof prof_b2176 300 5 --steps 10 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step vprof_fp8 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vprof_fp8 -- python benchmarks/value_training_benchmark.py --precision fp8 --steps 10
f=$(ls $O/vprof_fp8/*/*kernel_trace.csv 2>/dev/null | head -1)
if [ -n "$f" ]; then python3 scripts/timeline.py "$f" 10 > $O/vprof_fp8.timeline.txt 2>&1; head -25 $O/vprof_fp8.timeline.txt; rm -f "$f"; fi
grep -h '"value"' $O/bench*.log $O/value_*.log | cut -c1-220
