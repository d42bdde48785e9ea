#!/bin/bash
# Small batches after the reduce-tail fix: B = 16 / 32 / 64 / 128 and the B = 16 step timeline.
O=gpurun_out/r6/small
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
for B in 16 32 64 128; do
  step b${B}_r1 120 python bench.py --gpus 1 --batch $B --steps 300 --warmup 50
  step b${B}_r2 120 python bench.py --gpus 1 --batch $B --steps 300 --warmup 50
done
prof prof16 300 50 --batch 16 --steps 300 --warmup 50
for f in $O/b*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done
