#!/bin/bash
# 192-wide fp8 forward (policy): staged byte outputs with 8-wave workgroups (lab 7) vs production
set -o pipefail
O=gpurun_out/r5/b49
mkdir -p $O
for out in fp8 both fp8mb; do
  P_C=192 P_OUT=$out P_VARIANTS=0,7 timeout -k 10 200 python -u scripts/r5/fp8_probe2.py > $O/c192_$out.log 2>&1 || exit 1
done
P_C=192 P_OUT=fp8 P_B=64 P_VARIANTS=0,7 timeout -k 10 200 python -u scripts/r5/fp8_probe2.py > $O/c192_fp8_b64.log 2>&1
