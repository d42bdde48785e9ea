#!/bin/bash
# fp8 wgrad (value layer, B = 1024) timing probes
set -o pipefail
mkdir -p gpurun_out/r5/b44
timeout -k 10 300 python -u scripts/r5/wgrad_fp8_probe.py > gpurun_out/r5/b44/probe.log 2>&1
