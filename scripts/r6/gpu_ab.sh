#!/bin/bash
# Same-box A/B of the SL headline: the tree at this session's start (ab_base, a git worktree of
# 8950dc6, built in place) against HEAD, alternating, three runs each of the driver's bench command.
O=gpurun_out/r6/ab
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
for r in 1 2 3; do
  step base_r$r 300 bash -c "cd ab_base && python bench.py --gpus 1 --steps 20 --warmup 5"
  step head_r$r 300 python bench.py --gpus 1 --steps 20 --warmup 5
done
for f in $O/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
