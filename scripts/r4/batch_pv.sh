#!/bin/bash
# Round 4 batch PV: PMC of the fp8 value-training step (B = 1024).
O=gpurun_out/r4_pv
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step pmc_value 600 bash scripts/r4/pmc_value.sh $O/pmc --precision fp8
