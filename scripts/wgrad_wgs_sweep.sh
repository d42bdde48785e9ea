#!/bin/bash
# wgrad split-K target (workgroups per launch) with the serial backward
set -e
o=gpurun_out/wgs
mkdir -p $o
for rep in 1 2; do
  for w in 256 512 768 1024; do
    echo "wgs $w" >> $o/sweep.txt
    timeout -k 10 150 python -u bench.py --steps 40 --warmup 8 --wgrad-wgs $w 2>/dev/null | cut -c1-140 >> $o/sweep.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1
