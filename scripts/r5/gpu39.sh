#!/bin/bash
# fp8 160-wide forward timing probes (lab): both outputs, and the training forward's e4m3 + bitmask
set -o pipefail
mkdir -p gpurun_out/r5/b39

P_OUT=fp8mb timeout -k 10 300 python -u scripts/r5/fp8_probe2.py > gpurun_out/r5/b39/probe_fp8mb.log 2>&1
