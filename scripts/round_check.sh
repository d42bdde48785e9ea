#!/bin/bash
# One GPU call that checks the committed tree end to end: GPU tests, smoke, the
# default bench, and a kernel-trace profile of the bench step (scripts/profile_step.sh).
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rc_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/rc_tests.log; exit 1; }
tail -1 gpurun_out/rc_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc_smoke.log 2>&1
tail -1 gpurun_out/rc_smoke.log
timeout -k 10 180 python bench.py > gpurun_out/rc_bench.log 2>&1
tail -1 gpurun_out/rc_bench.log
timeout -k 10 180 bash scripts/profile_step.sh gpurun_out/prof6 --steps 20 --warmup 15 > gpurun_out/prof6.log 2>&1
f=$(find gpurun_out/prof6 -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py $f 5 > gpurun_out/timeline6.txt
cp $(find gpurun_out/prof6 -name "*kernel_stats.csv" | head -1) gpurun_out/kstats6.csv
cat gpurun_out/timeline6.txt
