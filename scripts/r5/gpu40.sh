#!/bin/bash
# fp8 160-wide forward: offset table (lab 132), LDS-staged byte outputs (164), both (196)
set -o pipefail
mkdir -p gpurun_out/r5/b40
P_VARIANTS=0,132,164,196 P_OUT=fp8mb timeout -k 10 300 python -u scripts/r5/fp8_probe2.py > gpurun_out/r5/b40/fp8mb.log 2>&1 &&
P_VARIANTS=0,132,164,196 timeout -k 10 300 python -u scripts/r5/fp8_probe2.py > gpurun_out/r5/b40/both.log 2>&1
