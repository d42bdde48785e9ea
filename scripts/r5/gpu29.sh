#!/bin/bash
# final-ish tree: full GPU suite, SL sweep, smoke
O=gpurun_out/r5/b29
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -E "passed|failed" $O/suite.log | tail -2
grep -q " passed" $O/suite.log && ! grep -q " failed" $O/suite.log || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for B in 1 8 16 32 64 128; do
  step sl$B 300 python -u bench.py --batch $B --steps 200 --warmup 20
done
for f in $O/sl*.log; do grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['host_ms_per_step'])"; done
