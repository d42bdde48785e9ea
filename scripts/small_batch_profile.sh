#!/bin/bash
# Small-batch SL step: eager/graph positions/s at B = 16/64/256, then a rocprofv3
# kernel trace of the eager B = 16, B = 256 and B = 2176 steps for per-kernel times and the serial tail.
set -e
O=${OUT:-gpurun_out/smallb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/graph_step_benchmark.py --batches ${BATCHES:-16,64,256} --steps 100 --warmup 10 | tee $O/graph_step.jsonl
for b in ${PROF_BATCHES:-16 256 2176}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$b -o run -- python3 bench.py --batch $b --steps 20 --warmup 5 > $O/bench$b.log 2>&1
  python scripts/timeline.py $O/p$b/run_kernel_trace.csv 5 > $O/timeline$b.txt
  rm -f $O/p$b/run_kernel_trace.csv  # large; the timeline keeps what is needed
  head -30 $O/timeline$b.txt
done
