#!/bin/bash
# small-batch sweep (merged reduce A/B) + the final-tree checks, one call
bash scripts/r6/gpu_b4.sh
rc=$?
[ $rc -ge 124 ] && exit $rc
bash scripts/r6/gpu_final.sh
