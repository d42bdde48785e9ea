#!/bin/bash
# coalesced wgrad reduce: tests, SL A/B (small-batch wgrad plan on / off, 256 / 512 WGs), B = 16 trace, bench
O=gpurun_out/r5/b27
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step test 600 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py tests/test_determinism_gpu.py tests/test_conv160.py -x -q --timeout 120 --timeout-method thread
grep -E "passed|failed" $O/test.log | tail -2
grep -q " passed" $O/test.log && ! grep -q "failed" $O/test.log || exit 1
for B in 16 32 8; do
  step new$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
  step old$B 300 env AGK_TMP_WGRAD_SMALL_MAX_M=0 python -u bench.py --batch $B --steps 300 --warmup 20
  step new512_$B 300 python -u bench.py --batch $B --steps 300 --warmup 20 --wgrad-wgs 512
done
for f in $O/new*.log $O/old*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
prof prof_sl16 300 40 --batch 16 --steps 40 --warmup 10
step bench_default 600 python -u bench.py
grep -h '^{' $O/bench_default.log | cut -c1-200
prof prof_b2176 600 10 --steps 10 --warmup 5
