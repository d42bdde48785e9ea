#!/bin/bash
# A/B of forward/dgrad tilings on the value bench (alternating runs):
# usage scripts/tile_ab_value.sh "384 385" [reps] [extra value-bench args]
set -e
o=gpurun_out/tile_ab
mkdir -p $o
arms=${1:-"384 385"}
reps=${2:-3}
for rep in $(seq $reps); do
  for t in $arms; do
    echo "tile $t $3" >> $o/value.txt
    timeout -k 10 150 python -u benchmarks/value_training_benchmark.py --steps 100 --conv-tile $t $3 2>/dev/null | cut -c1-110 >> $o/value.txt
  done
done
