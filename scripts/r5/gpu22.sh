#!/bin/bash
# SL at B = 16 / 32: eager vs graph-captured step (serial capture / two-stream capture)
O=gpurun_out/r5/b22
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
for B in 16 32; do
  step eager$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
  step graph$B 300 python -u bench.py --batch $B --steps 300 --warmup 20 --graph
  step graphov$B 300 env ALPHAGO_AMD_GRAPH_OVERLAP=1 python -u bench.py --batch $B --steps 300 --warmup 20 --graph
done
for f in $O/*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
