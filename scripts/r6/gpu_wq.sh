#!/bin/bash
# fp8 weight pack (256 blocks per job) and weight scales (16 loads in flight): value step timeline.
O=gpurun_out/r6/wq
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
step tests 600 python -u -m pytest tests/test_fp8_inference.py tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fp8"
step value_fp8_r1 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
step value_fp8_r2 300 python -u benchmarks/value_training_benchmark.py --precision fp8 --steps 30
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step vprof_fp8 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vprof_fp8 -- python benchmarks/value_training_benchmark.py --precision fp8 --steps 10
f=$(ls $O/vprof_fp8/*/*kernel_trace.csv 2>/dev/null | head -1)
if [ -n "$f" ]; then python3 scripts/timeline.py "$f" 10 > $O/vprof_fp8.timeline.txt 2>&1; grep -E "span|weight|pack" $O/vprof_fp8.timeline.txt; rm -f "$f"; fi
grep -h '"value"' $O/value_*.log | cut -c1-200
