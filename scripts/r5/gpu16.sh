#!/bin/bash
# weight-stationary probes (lab tiles 41..47: no loads / no MFMA / no epilogue) at B = 1 / 8 / 16;
# genmove from the empty board (the random net's edge-heavy games) with the ladder cache on / off
O=gpurun_out/r5/b16
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step probes 300 env WS_WIDTHS=192 WS_BATCHES=1,4,8,16,32 WS_TILES=0,40,41,42,43,44,46,47 python -u scripts/r5/ws_bench.py
grep '"C"' $O/probes.log
step gm_cache 600 python -u benchmarks/genmove_benchmark.py --leaves 32 --moves 10 --ladder-cache 1
step gm_nocache 600 python -u benchmarks/genmove_benchmark.py --leaves 32 --moves 10 --ladder-cache 0
grep -h ms_per $O/gm_*.log | cut -c1-300
