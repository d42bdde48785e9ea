#!/bin/bash
# Same-box A/B of two builds of the production library: alphago_amd/_ab_old/_hip_kernels.so (A, old)
# vs alphago_amd/_ab_old/_hip_kernels_new.so (B, new), each bench in its own process.
# Optional: TESTS="pytest args" run first on the new build.
set -e
O=gpurun_out/soab
mkdir -p $O
export PYTHONPATH=$PWD
cp alphago_amd/_ab_old/_hip_kernels_new.so alphago_amd/_hip_kernels.so
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp alphago_amd/_ab_old/_hip_kernels.so alphago_amd/_hip_kernels.so; else cp alphago_amd/_ab_old/_hip_kernels_new.so alphago_amd/_hip_kernels.so; fi
    timeout -k 10 200 python3 ${BENCH:-bench.py} --steps 20 --warmup 5 > $O/$v.json 2> $O/$v.err
    echo "$r $v $(python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
cp alphago_amd/_ab_old/_hip_kernels_new.so alphago_amd/_hip_kernels.so
