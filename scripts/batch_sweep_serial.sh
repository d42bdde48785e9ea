#!/bin/bash
# SL bench per-GPU batch sweep with the serial backward (alternating repetitions)
set -e
o=gpurun_out/bsw
mkdir -p $o
for rep in 1 2; do
  for b in 2176 3264 4352; do
    echo "batch $b" >> $o/sweep.txt
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 6 --batch $b 2>/dev/null | cut -c1-140 >> $o/sweep.txt
  done
done
