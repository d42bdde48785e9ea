#!/bin/bash
# Small-batch wgrad split depth: minimum 32-pixel stages per split (ops.WGRAD_MIN_STAGES) at B = 16 / 32,
# two alternating passes.
O=gpurun_out/r6/stages
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
for r in 1 2; do
  for B in 16 32; do
    for st in 4 8 16 32; do
      ALPHAGO_AMD_WGRAD_MIN_STAGES=$st step b${B}_s${st}_r$r 120 python bench.py --gpus 1 --batch $B --steps 300 --warmup 50
    done
  done
done
for f in $O/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done
