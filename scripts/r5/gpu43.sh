#!/bin/bash
# value fp8 training step after the 4-wave / staged-output fp8 conv: kernel timeline + MFMA-busy PMC
set -o pipefail
O=gpurun_out/r5/b43
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -- python3 benchmarks/value_training_benchmark.py --precision fp8 --steps 20 --warmup 5 --data random > $O/prof.log 2>&1 &&
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1) && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/p1 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -- python3 benchmarks/value_training_benchmark.py --precision fp8 --steps 8 --warmup 3 --pool 8192 --heldout 1024 > $O/p1.log 2>&1
rm -f $O/prof/*/*.csv.gz 2>/dev/null
du -sh $O
