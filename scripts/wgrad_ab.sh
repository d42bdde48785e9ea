#!/bin/bash
# A/B of the wgrad LDS-DMA issue (0 = burst, 5 = spread) on the SL bench and the
# value bench, alternating runs: usage scripts/wgrad_ab.sh [reps]
set -e
o=gpurun_out/wgrad_ab
mkdir -p $o
reps=${1:-3}
for rep in $(seq $reps); do
  for v in 0 5; do
    echo "wgrad-variant $v" >> $o/policy.txt
    timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 --wgrad-variant $v 2>/dev/null | cut -c1-140 >> $o/policy.txt
  done
done
