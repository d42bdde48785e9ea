#!/bin/bash
# Round-3 GPU check of the committed tree: full GPU suite, smoke, driver-shaped bench, and
# rocprofv3 kernel-trace profiles of the SL step and of the fp8 value step.  Output: gpurun_out/r3c/
set -e
O=gpurun_out/r3c
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err
tail -1 $O/bench1.json | cut -c1-300
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sl -- python3 bench.py --steps 20 --warmup 15 > $O/prof_sl.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_value -- python3 benchmarks/value_training_benchmark.py --steps 20 --warmup 5 > $O/prof_value.log 2>&1
f=$(find $O/prof_sl -name "*kernel_stats.csv" | head -1); cp $f $O/sl_kernel_stats.csv
f=$(find $O/prof_value -name "*kernel_stats.csv" | head -1); cp $f $O/value_kernel_stats.csv
f=$(find $O/prof_sl -name "*kernel_trace.csv" | head -1); python3 scripts/timeline.py $f 5 > $O/sl_timeline.txt
head -30 $O/sl_timeline.txt
