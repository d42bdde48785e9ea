#!/bin/bash
# bench.py per-GPU batch sweep at the round-3 head (same box, two passes)
set -e
O=gpurun_out/bs3
mkdir -p $O
export PYTHONPATH=$PWD
for pass in 1 2; do
  for b in 2176 3264 4352; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --batch $b > $O/b$b.json 2> $O/b$b.err
    echo "pass $pass B=$b $(python3 -c "import json; d=json.loads(open('$O/b$b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('top1_acc'))")"
  done
done
