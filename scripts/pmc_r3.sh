#!/bin/bash
# Round-3 PMC passes on the production conv kernels (fwd, bitmask dgrad, wgrad) and the SL wgrad shapes.
set -e
bash scripts/pmc_conv.sh > /dev/null
OUT=gpurun_out/wpmc bash scripts/probes/wgrad_pmc.sh > gpurun_out/wpmc_summary.txt 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt
cat gpurun_out/pmc_summary.txt | grep -E "==|mfma_busy|wait_any|clock"
cat gpurun_out/wpmc_summary.txt | grep -E "==|mfma_busy|wait_any|clock"
