#!/bin/bash
# final tree after the fp8 value-width kernels: full GPU suite, smoke, default bench, value fp8/bf16
# benchmarks, value fp8 step timeline
O=gpurun_out/r5/b47
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
grep -E "passed|failed" $O/suite.log | tail -2
grep -q " passed" $O/suite.log && ! grep -q " failed" $O/suite.log || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python -u bench.py
grep -h '^{' $O/bench.log | cut -c1-300
step value_fp8 400 python -u benchmarks/value_training_benchmark.py --precision fp8
step value_bf16 400 python -u benchmarks/value_training_benchmark.py --precision bf16
step vprof 300 rocprofv3 --kernel-trace --output-format csv -d $O/vprof -- python3 benchmarks/value_training_benchmark.py --precision fp8 --steps 20 --warmup 5 --data random
f=$(ls $O/vprof/*/*kernel_trace.csv 2>/dev/null | head -1)
if [ -n "$f" ]; then python3 scripts/timeline.py "$f" 5 > $O/vprof.timeline.txt 2>&1; rm -f "$f"; fi
head -8 $O/vprof.timeline.txt
