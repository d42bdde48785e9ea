#!/bin/bash
# Round 4 batch E: fp8 training diagnosis; 12-wave layer-0 wgrad (variant 10) tests, A/B and trace.
# Output: gpurun_out/r4_e/
O=gpurun_out/r4_e
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step train_diag 200 python3 -u scripts/r4/fp8_train_diag.py
step thin 200 python3 -u -m pytest tests/test_hip_kernels.py -k "thin_input or small_batch" -m gpu -q --timeout 120 --timeout-method thread
step ab_w6 200 python3 bench.py --steps 100 --warmup 20
step ab_w12 200 env ALPHAGO_AMD_WGRAD0_WAVES=12 python3 bench.py --steps 100 --warmup 20
step ab_w6b 200 python3 bench.py --steps 100 --warmup 20
step ab_w12b 200 env ALPHAGO_AMD_WGRAD0_WAVES=12 python3 bench.py --steps 100 --warmup 20
export ALPHAGO_AMD_WGRAD0_WAVES=12
step prof 300 bash scripts/profile_step.sh $O/prof --steps 20 --warmup 5
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1; head -20 $O/timeline.txt
