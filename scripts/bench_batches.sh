#!/bin/bash
# bench.py at several per-GPU batch sizes (after one warm-up run)
export PYTHONPATH=$PWD
timeout -k 10 120 python bench.py --steps 10 --warmup 10 > /dev/null 2>&1
for b in ${@:-1088 2176 3264 1088 2176 3264}; do
  timeout -k 10 240 python bench.py --steps 40 --warmup 20 --batch $b 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('batch', $b, d['value'], d['ms_per_step'])"
done
