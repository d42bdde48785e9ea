#!/bin/bash
# PMC pass over the value-training step (160-wide tiles): MFMA busy, wave waits,
# clock; one counter pass per rocprofv3 run (gpurun rules), kernel trace in p1.
set -e
o=${1:-gpurun_out/pmcv}
mkdir -p $o
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $R/$o/value/p1 -o run -- python3 $R/benchmarks/value_training_benchmark.py --precision bf16 --steps 3 --warmup 2 > $R/$o/p1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/$o/value/runc -o run -- python3 $R/benchmarks/value_training_benchmark.py --precision bf16 --steps 3 --warmup 2 > $R/$o/p2.log 2>&1
