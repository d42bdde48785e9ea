#!/bin/bash
# Round 4 batch C: fp8 value-trainer failures at width 160 with 32- vs 64-channel weight chunks, the
# rewritten sgd_pack, the packed-tap trainer test, small-batch tests, kernel trace of the B = 16 step.
# Output: gpurun_out/r4_c/
O=gpurun_out/r4_c
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
FP8T="tests/test_fp8_inference.py::test_fp8_backward_12_layer_trunk_matches_exact_backward tests/test_fp8_inference.py::test_fp8_value_training_tracks_bf16"
step fp8_cw32 300 python3 -u -m pytest $FP8T -m gpu -q -s --timeout 120 --timeout-method thread
step fp8_cw64 300 env ALPHAGO_AMD_FP8_CW32=0 python3 -u -m pytest $FP8T -m gpu -q -s --timeout 120 --timeout-method thread
step trainer 300 python3 -u -m pytest tests/test_hip_trainer.py tests/test_hip_kernels.py -k "fused_sgd_pack or packed_tap or small_batch" -m gpu -q --timeout 120 --timeout-method thread
step ab_new 200 python3 bench.py --steps 100 --warmup 20
step ab_fused0 200 env ALPHAGO_AMD_FUSED_UPDATE=0 python3 bench.py --steps 100 --warmup 20
step prof16 200 bash scripts/profile_step.sh $O/prof16 --batch 16 --steps 200 --warmup 50 --pool 8192
f=$(ls $O/prof16/*/*kernel_trace.csv $O/prof16/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 200 > $O/timeline16.txt 2>&1; head -40 $O/timeline16.txt
step prof 300 bash scripts/profile_step.sh $O/prof --steps 20 --warmup 5
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1; head -12 $O/timeline.txt
