#!/bin/bash
# Value-net training step timelines (fp8 and bf16, B = 1024).
O=gpurun_out/r6/vprof
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for p in fp8 bf16; do
  step prof_$p 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$p -- python benchmarks/value_training_benchmark.py --precision $p --steps 10
  f=$(ls $O/prof_$p/*/*kernel_trace.csv 2>/dev/null | head -1)
  if [ -n "$f" ]; then
    python3 scripts/timeline.py "$f" 10 > $O/prof_$p.timeline.txt 2>&1
    head -30 $O/prof_$p.timeline.txt
    rm -f "$f"
  fi
done
