#!/bin/bash
# weight-stationary probes incl. no weight loads (bit 8); rocprof kernel trace of the B = 16 SL step
O=gpurun_out/r5/b17
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step probes 300 env WS_WIDTHS=192 WS_BATCHES=1,8,16 WS_TILES=40,47,48,50,55 python -u scripts/r5/ws_bench.py
grep '"C"' $O/probes.log
prof prof_sl16 300 40 --batch 16 --steps 40 --warmup 10
