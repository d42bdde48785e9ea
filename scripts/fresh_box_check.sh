#!/bin/bash
# First-process-on-a-fresh-box diagnosis (VERDICT r1 "fresh-box deficit"):
#   1. the EXACT driver bench command as the first GPU process, under rocprofv3 --kernel-trace
#   2. the same command twice more without the profiler
#   3. GPU clocks / power / activity sampled with amd-smi (1 Hz) for the whole call
# Output: gpurun_out/fresh/
set -e
O=gpurun_out/fresh
mkdir -p $O
export PYTHONPATH=$PWD
amd-smi static -g 0 > $O/smi_static.txt 2>&1 || true
( while true; do date +%s.%N; amd-smi metric -g 0 2>&1 | grep -iE "CLK|POWER|GFX_ACTIVITY|TEMP|HOTSPOT|SOCKET|UMC|MEM_ACT" | head -40; echo ---; sleep 1; done ) > $O/smi_monitor.txt 2>&1 &
MON=$!
trap "kill $MON 2>/dev/null || true" EXIT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
date +%s.%N > $O/t_prof_start
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err
date +%s.%N > $O/t_prof_end
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench2.json 2> $O/bench2.err
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench3.json 2> $O/bench3.err
timeout -k 10 120 python3 bench.py --gpus 1 --steps 100 --warmup 5 > $O/bench4.json 2> $O/bench4.err
cat $O/bench_prof.json $O/bench2.json $O/bench3.json $O/bench4.json
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kstats.csv
