#!/bin/bash
# Round 4 batch H: layer-0 wgrad variants (10 = 12 waves, 11 = 4-slot ring, 12 = both) tests + A/B +
# trace; 32-pixel forward tiles (36 / 37) at B = 16; the reworked fp8 tests.  Output: gpurun_out/r4_h/
O=gpurun_out/r4_h
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step tests 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_fp8_inference.py -k "thin_input or small_batch or tile_variants or ring_5x5 or bitmask or fp8_value_training or fp8_backward" -m gpu -q -s --timeout 150 --timeout-method thread
for V in 0 11 12 0 11; do
  step ab_v${V}_$RANDOM 200 env ALPHAGO_AMD_WGRAD0_VARIANT=$V python3 bench.py --steps 100 --warmup 20
done
for T in 64 36 37 65; do
  step sl16_t$T 120 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192 --conv-tile $T
done
export ALPHAGO_AMD_WGRAD0_VARIANT=11
step prof 300 bash scripts/profile_step.sh $O/prof --steps 20 --warmup 5
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1; head -8 $O/timeline.txt; tail -3 $O/timeline.txt
export ALPHAGO_AMD_WGRAD0_VARIANT=0
step prof36 200 bash scripts/profile_step.sh $O/prof36 --batch 16 --steps 200 --warmup 50 --pool 8192 --conv-tile 36
f=$(ls $O/prof36/*/*kernel_trace.csv $O/prof36/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 200 > $O/timeline36.txt 2>&1; head -8 $O/timeline36.txt
