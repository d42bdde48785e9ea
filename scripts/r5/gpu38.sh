#!/bin/bash
# full GPU suite + smoke + default bench on the current tree
O=gpurun_out/r5/b38
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
grep -E "passed|failed" $O/suite.log | tail -2
grep -q " passed" $O/suite.log && ! grep -q " failed" $O/suite.log || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python -u bench.py
grep -h '^{' $O/bench.log | cut -c1-300
