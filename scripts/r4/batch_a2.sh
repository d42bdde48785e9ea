#!/bin/bash
# Round 4 batch A2 (after the conv_wgrad variant-9 op fix and the sgd_pack rewrite): GPU tests of the
# files touched this round, update-path A/B, small-batch kernels and SL steps, kernel trace.
# Output: gpurun_out/r4_a2/
O=gpurun_out/r4_a2
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step kernels 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_conv160.py tests/test_hip_trainer.py tests/test_fp8_inference.py tests/test_lockstep.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread
step ab_new 200 python3 bench.py --steps 100 --warmup 20
step ab_fused0 200 env ALPHAGO_AMD_FUSED_UPDATE=0 python3 bench.py --steps 100 --warmup 20
step kbench 200 python3 -u scripts/r4/small_batch_kbench.py 1 4 16 64 256
step sl_b16 120 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192
step sl_b16_ring0 120 env ALPHAGO_AMD_WGRAD_RING=0 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192
step sl_b16_t65 120 python3 bench.py --batch 16 --steps 300 --warmup 50 --pool 8192 --conv-tile 65
step prof 300 bash scripts/profile_step.sh $O/prof --steps 20 --warmup 5
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1; head -30 $O/timeline.txt
