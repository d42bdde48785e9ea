#!/bin/bash
# small-batch wgrad plan (64 x 64 tap-merged tiles): tests, SL A/B at B = 8 / 16 / 32, graph mode
O=gpurun_out/r5/b26
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step wg_test 300 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -x -q --timeout 120 --timeout-method thread -k "conv_wgrad or weight_stationary or small_batch or splitk"
grep -E "passed|failed" $O/wg_test.log | tail -2
grep -q " passed" $O/wg_test.log && ! grep -q "failed" $O/wg_test.log || exit 1
for B in 16 32 8; do
  step new$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
  step old$B 300 env AGK_TMP_WGRAD_SMALL_MAX_M=0 python -u bench.py --batch $B --steps 300 --warmup 20
  step new512_$B 300 python -u bench.py --batch $B --steps 300 --warmup 20 --wgrad-wgs 512
  step graph$B 300 python -u bench.py --batch $B --steps 300 --warmup 20 --graph
done
for f in $O/new*.log $O/old*.log $O/graph*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
prof prof_sl16 300 40 --batch 16 --steps 40 --warmup 10
