#!/bin/bash
# fp8 160-wide forward: LDS-staged byte outputs (164), 4-wave workgroups two per CU (228), both (292)
set -o pipefail
mkdir -p gpurun_out/r5/b41
P_VARIANTS=0,164,228,292 P_OUT=fp8mb timeout -k 10 300 python -u scripts/r5/fp8_probe2.py > gpurun_out/r5/b41/fp8mb.log 2>&1 &&
P_VARIANTS=0,164,228,292 timeout -k 10 300 python -u scripts/r5/fp8_probe2.py > gpurun_out/r5/b41/both.log 2>&1
