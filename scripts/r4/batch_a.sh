#!/bin/bash
# Round 4 batch A: GPU test files touched this round, small-batch kernel timings, SL step at
# B = 2176 / 16 / 64 / 256, in-step kernel trace.  Output: gpurun_out/r4_a/
O=gpurun_out/r4_a
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step kernels 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_conv160.py tests/test_hip_trainer.py tests/test_fp8_inference.py tests/test_lockstep.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench2176 240 python3 bench.py --gpus 1 --steps 20 --warmup 5
# same-box A/Bs of this round's bench-path changes (each arm 100 steps)
step ab_new 200 python3 bench.py --steps 100 --warmup 20
step ab_pk0 200 env ALPHAGO_AMD_PK=0 python3 bench.py --steps 100 --warmup 20
step ab_fused0 200 env ALPHAGO_AMD_FUSED_UPDATE=0 python3 bench.py --steps 100 --warmup 20
step ab_occ3 200 env AGK_WGRAD0_OCC3=1 python3 bench.py --steps 100 --warmup 20
step ab_new2 200 python3 bench.py --steps 100 --warmup 20
step kbench 200 python3 -u scripts/r4/small_batch_kbench.py 1 4 16 64 256
for B in 16 64 256; do
  for T in 0 65; do
    step sl_b${B}_t${T} 120 python3 bench.py --batch $B --steps 200 --warmup 50 --conv-tile $T --pool 8192
  done
done
step prof 300 bash scripts/profile_step.sh $O/prof --steps 20 --warmup 5
f=$(ls $O/prof/*/*kernel_trace.csv $O/prof/*kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 scripts/timeline.py "$f" 5 > $O/timeline.txt 2>&1; head -30 $O/timeline.txt
