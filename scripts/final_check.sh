#!/bin/bash
# Round-end rehearsal in the driver's order: the driver's bench command as the FIRST GPU process
# on a fresh box, then the full GPU suite, smoke, and the bench again.  Output: gpurun_out/final2/
set -e
O=gpurun_out/final2
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err
tail -1 $O/bench1.json | cut -c1-220
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench2.json 2> $O/bench2.err
tail -1 $O/bench2.json | cut -c1-220
