#!/bin/bash
# Round-6 batch 3: fp8 underflow guard -- SL fp8-forward (round to nearest) over 5 seeds vs bf16 and the
# unguarded scale, then value precision parity on 4x the round-5 positions.
set -o pipefail
O=gpurun_out/r6/fp8
mkdir -p $O
export PYTHONUNBUFFERED=1
for s in 0 1 2 3 4; do
  timeout -k 10 240 python scripts/sl_teacher_accuracy.py /tmp/slacc_$s --positions 131072 --epochs 4 --seed $s \
    --arms hip-bf16,hip-fp8fwd,hip-fp8fwd-noguard >> $O/sl_fp8_guard.jsonl 2> $O/sl_fp8_guard_$s.err || exit 1
  tail -1 $O/sl_fp8_guard.jsonl
done
timeout -k 10 1000 python -u scripts/value_fp8_parity.py $O/parity_value_4x.json --task material \
  --positions 262144 --epochs 4 --arms torch-fp32,hip-bf16,hip-fp8 --optimizer adam --lr 0.0003 --decay 0.005 \
  --seeds 5 > $O/parity_value_4x.log 2>&1
rc=$?
tail -5 $O/parity_value_4x.log
exit $rc
