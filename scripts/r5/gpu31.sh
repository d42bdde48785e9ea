#!/bin/bash
O=gpurun_out/r5/b31
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step red 300 python -u scripts/r5/reduce_bench.py
grep nsplit $O/red.log
for B in 8 16 32; do
  step ov0_$B 300 env ALPHAGO_AMD_OVERLAP=0 python -u bench.py --batch $B --steps 300 --warmup 20
  step ov1_$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
done
for f in $O/ov*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
