#!/bin/bash
# batches 5 + 7 in one call (box acquisition is the bottleneck this round)
bash scripts/r6/gpu_b5.sh
rc=$?
[ $rc -ge 124 ] && exit $rc
bash scripts/r6/gpu_b7.sh
