#!/bin/bash
# batch 9 (fp32 arm of the self-play value run) + batch 4 (small-batch sweep), one call
bash scripts/r6/gpu_b9.sh
rc=$?
[ $rc -ge 124 ] && exit $rc
bash scripts/r6/gpu_b4.sh
