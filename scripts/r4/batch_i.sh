#!/bin/bash
# Round 4 batch I: wgrad unit pipelining (layer 0: variants 11 / 12 / 15; 3x3: ALPHAGO_AMD_WGRAD_UP=1 ->
# variant 14): tests, same-box A/B (100 steps each, interleaved), kernel trace.  Output: gpurun_out/r4_i/
O=gpurun_out/r4_i
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_hip_kernels.py -k "thin_input or test_conv_wgrad" -m gpu -q --timeout 150 --timeout-method thread
ab() { step ab_$1_$2_$RANDOM 200 env ALPHAGO_AMD_WGRAD0_VARIANT=$1 ALPHAGO_AMD_WGRAD_UP=$2 python3 bench.py --steps 100 --warmup 20; }
ab 0 0; ab 11 0; ab 12 0; ab 15 0; ab 0 1; ab 11 1; ab 0 0; ab 11 1
export ALPHAGO_AMD_WGRAD0_VARIANT=11 ALPHAGO_AMD_WGRAD_UP=1
step prof 300 bash scripts/profile_step.sh $O/prof --steps 20 --warmup 5
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1; head -8 $O/timeline.txt; tail -3 $O/timeline.txt
export ALPHAGO_AMD_WGRAD0_VARIANT=12 ALPHAGO_AMD_WGRAD_UP=0
step prof12 300 bash scripts/profile_step.sh $O/prof12 --steps 20 --warmup 5
f=$(ls $O/prof12/*/*kernel_trace.csv $O/prof12/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline12.txt 2>&1; head -6 $O/timeline12.txt
