#!/bin/bash
# host profile of the B = 16 eager step; WS on / off in training at B = 16 / 32; the default bench
O=gpurun_out/r5/b24
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step cprof16 300 python -u scripts/r5/step_cprofile.py 16
head -45 $O/cprof16.log | tail -32
for B in 16 32; do
  step ws1_$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
  step ws0_$B 300 env ALPHAGO_AMD_WS=0 python -u bench.py --batch $B --steps 300 --warmup 20
done
step bench_default 600 python -u bench.py
for f in $O/ws*.log $O/bench_default.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'], d.get('hbm_peak_gib_per_rank'), d.get('pool_build_s'))"; done
