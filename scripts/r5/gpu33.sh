#!/bin/bash
O=gpurun_out/r5/b33
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step test 500 python -u -m pytest tests/test_distributed_gpu.py tests/test_hip_trainer.py -x -v --timeout 150 --timeout-method thread
grep -E "passed|failed" $O/test.log | tail -2
grep -q " passed" $O/test.log && ! grep -q " failed" $O/test.log || exit 1
for B in 1 4 8 16 24 32; do
  step sl$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
done
for f in $O/sl*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
step slacc 600 python -u scripts/sl_teacher_accuracy.py $O/slacc --positions 131072 --epochs 4 --arms hip-bf16,hip-fp8fwd
tail -1 $O/slacc.log | cut -c1-600
step slacc_sr 600 env ALPHAGO_AMD_FP8_SR=1 python -u scripts/sl_teacher_accuracy.py $O/slacc_sr --positions 131072 --epochs 4 --arms hip-fp8fwd
tail -1 $O/slacc_sr.log | cut -c1-400
