#!/bin/bash
# Round-6 evidence call 1: SL net on the teacher pool -> RL (100 x 512 games) -> RL vs SL match.
set -o pipefail
O=gpurun_out/r6/ev
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/r6/evidence.py sl $O --positions 262144 --epochs 6 --batch 256 --lr 0.05 > $O/sl.log 2>&1 &&
timeout -k 10 600 python scripts/r6/evidence.py rl $O --games 512 --iterations 100 --save-every 10 --lr 0.03 --batch 1024 > $O/rl.log 2>&1 &&
timeout -k 10 240 python scripts/r6/evidence.py match $O --games 1000 > $O/match.log 2>&1
rc=$?
tail -3 $O/*.log
exit $rc
