#!/bin/bash
# WS ring: two-stage row prefetch + batched prologue: tests, per-layer times, probes, latency, SL
O=gpurun_out/r5/b36
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step ws_test 300 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_trainer.py -x -q --timeout 120 --timeout-method thread -k "weight_stationary or small_batch"
grep -E "passed|failed" $O/ws_test.log | tail -2
grep -q " passed" $O/ws_test.log && ! grep -q " failed" $O/ws_test.log || exit 1
step ws_bench 300 env WS_BATCHES=1,4,8,16,32 python -u scripts/r5/ws_bench.py
grep '"C"' $O/ws_bench.log
step probes 300 env WS_WIDTHS=192 WS_BATCHES=1,16 WS_TILES=40,1014 python -u scripts/r5/ws_bench.py
grep '"C"' $O/probes.log
step fwd_lat 300 python -u benchmarks/forward_latency_benchmark.py --batches 1,4,8,16,32 --iters 30
grep bf16 $O/fwd_lat.log
for B in 1 8 16; do
  step sl$B 300 python -u bench.py --batch $B --steps 300 --warmup 20
done
for f in $O/sl*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
