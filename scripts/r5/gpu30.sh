#!/bin/bash
# prebuilt launch lists: trainer tests, SL sweep, B = 16 host profile
O=gpurun_out/r5/b30
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step test 600 python -u -m pytest tests/test_hip_trainer.py tests/test_determinism_gpu.py tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread
grep -E "passed|failed" $O/test.log | tail -2
grep -q " passed" $O/test.log && ! grep -q " failed" $O/test.log || exit 1
for B in 1 8 16 32 64; do
  step sl$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
done
for f in $O/sl*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
