#!/bin/bash
# Round 4 batch T: PMC passes of the SL step at B = 2176 (per kernel: MFMA busy, waits, L2 hits) and of
# the stand-alone wgrad shapes (r3 probe).  Output: gpurun_out/r4_t/
O=gpurun_out/r4_t
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step pmc2176 600 bash scripts/r4/pmc_small.sh $O/pmc2176 2176 --pool 4096
step wpmc 600 env OUT=$O/wpmc bash scripts/probes/wgrad_pmc.sh
