#!/bin/bash
# weight-stationary probes: coalesced weight / activation loads (1016 / 1032 / 1048)
O=gpurun_out/r5/b18
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step probes 300 env WS_WIDTHS=192 WS_BATCHES=1,4,8,16,32 WS_TILES=40,1008,1016,1032,1048 python -u scripts/r5/ws_bench.py
grep '"C"' $O/probes.log
