#!/bin/bash
# Round 4 batch P: RL iteration with 2048-position REINFORCE chunks (native driver), the fp8 / bf16 value
# step kernel traces.  Output: gpurun_out/r4_p/
O=gpurun_out/r4_p
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
source scripts/r4/lib.sh
step rl 500 python3 -u benchmarks/rl_iteration_benchmark.py --games 20,512 --iterations 2 --records device --drivers native
for P in fp8 bf16; do
  step vprof_$P 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vprof_$P -- python3 benchmarks/value_training_benchmark.py --precision $P --steps 20 --warmup 5 --data random
  f=$(ls $O/vprof_$P/*/*kernel_trace.csv 2>/dev/null | head -1)
  if [ -n "$f" ]; then python3 scripts/timeline.py "$f" 5 > $O/vprof_$P.timeline.txt 2>&1; head -22 $O/vprof_$P.timeline.txt; rm -f "$f"; fi
done
