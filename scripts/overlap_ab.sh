#!/bin/bash
# A/B of the dgrad/wgrad two-stream overlap (and the fp8 dgrad) on one GPU:
# alternating runs so that clock/thermal drift hits both arms alike.
set -e
o=gpurun_out/ab
mkdir -p $o
for rep in 1 2 3; do
  for arm in "--overlap" ""; do
    echo "policy $arm" >> $o/policy.txt
    timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 $arm 2>/dev/null | cut -c1-140 >> $o/policy.txt
  done
  for arm in "--precision bf16 --overlap" "--precision bf16" "--precision fp8 --fp8-dgrad" "--precision fp8"; do
    echo "value $arm" >> $o/value.txt
    timeout -k 10 150 python -u benchmarks/value_training_benchmark.py --steps 100 $arm 2>/dev/null | cut -c1-110 >> $o/value.txt
  done
done
