#!/bin/bash
# fp8 weight scales with 16-B loads: test, value fp8 bench, step timeline
O=gpurun_out/r5/b52
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv160.py tests/test_fp8_inference.py
grep -q " passed" $O/tests.log && ! grep -q -E " failed| error" $O/tests.log || exit 1
step value_fp8 400 python -u benchmarks/value_training_benchmark.py --precision fp8
step vprof 300 rocprofv3 --kernel-trace --output-format csv -d $O/vprof -- python3 benchmarks/value_training_benchmark.py --precision fp8 --steps 20 --warmup 5 --data random
f=$(ls $O/vprof/*/*kernel_trace.csv 2>/dev/null | head -1)
if [ -n "$f" ]; then python3 scripts/timeline.py "$f" 5 > $O/vprof.timeline.txt 2>&1; rm -f "$f"; fi
head -14 $O/vprof.timeline.txt
