#!/bin/bash
# Round 4 combo: lockstep driver, then the small-batch check: kernel numerics (ring tiles, ring wgrad), kernel timings, SL step at
# B = 16 / 64 / 256 eager and graph.  Output: gpurun_out/r4_small/
set -e
bash scripts/r4/lockstep.sh
O=gpurun_out/r4_small
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py -k "small_batch or tile_variants or ring_5x5 or bitmask_dgrad or conv_wgrad or packed_taps" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 -u -m pytest tests/test_conv160.py -x -q --timeout 120 --timeout-method thread > $O/tests160.log 2>&1 || { tail -30 $O/tests160.log; exit 1; }
tail -2 $O/tests160.log
timeout -k 10 200 python3 -u scripts/r4/small_batch_kbench.py 1 4 16 64 256 > $O/kbench.jsonl 2> $O/kbench.err
cat $O/kbench.jsonl
for B in 16 64 256; do
  for T in 0 65; do
    timeout -k 10 120 python3 bench.py --batch $B --steps 200 --warmup 50 --conv-tile $T --pool 8192 > $O/sl_b${B}_t${T}.json 2> $O/sl_b${B}_t${T}.err
    tail -1 $O/sl_b${B}_t${T}.json | cut -c1-200
  done
done
