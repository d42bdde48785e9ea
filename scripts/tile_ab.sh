#!/bin/bash
# A/B of forward/dgrad tilings on the SL bench (alternating runs, so clock and
# thermal drift hit every arm alike): usage scripts/tile_ab.sh "0 385" [reps]
set -e
o=gpurun_out/tile_ab
mkdir -p $o
arms=${1:-"0 385"}
reps=${2:-3}
for rep in $(seq $reps); do
  for t in $arms; do
    echo "tile $t" >> $o/policy.txt
    timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 --conv-tile $t 2>/dev/null | cut -c1-140 >> $o/policy.txt
  done
done
