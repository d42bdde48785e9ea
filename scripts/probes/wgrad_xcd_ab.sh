#!/bin/bash
# Layer-0 wgrad: XCD-grouped kernel-row workgroups vs launch order (AGK_WGRAD_XCD=0), kernel trace + L2 hits.
set -e
export PYTHONPATH=$PWD TMPDIR=/tmp
OUT=${OUT:-gpurun_out/wxcd}
mkdir -p $OUT
for r in 1 2; do for x in 0 1; do
  AGK_WGRAD_XCD=$x timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/x$x/p1 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -- python3 scripts/probes/wgrad_pmc_one.py w0 > /dev/null 2>&1
  python3 scripts/pmc_summary.py $OUT | grep -A4 "== x$x" | head -5
  rm -rf $OUT/x$x
done; done
