#!/bin/bash
export PYTHONPATH=$PWD
for b in ${@:-1024 1536 2048 1024}; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --batch $b 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('batch', $b, d['value'], d['ms_per_step'])"
done
