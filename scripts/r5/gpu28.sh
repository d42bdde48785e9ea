#!/bin/bash
# small-batch wgrad plan at B = 24 .. 64 (one or two workgroups per CU) vs the per-tap plan
O=gpurun_out/r5/b28
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
for B in 24 32 48 64; do
  step old$B 300 env AGK_TMP_WGRAD_SMALL_MAX_M=0 python -u bench.py --batch $B --steps 300 --warmup 20
  step s1_$B 300 env AGK_TMP_WGRAD_SMALL_MAX_M=100000 python -u bench.py --batch $B --steps 300 --warmup 20
  step s2_$B 300 env AGK_TMP_WGRAD_SMALL_MAX_M=100000 AGK_TMP_WGRAD_SMALL_PERCU=2 python -u bench.py --batch $B --steps 300 --warmup 20
done
for f in $O/*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
step fp8probe 300 python -u scripts/r5/fp8_probe.py
cat $O/fp8probe.log | grep us_per
