#!/bin/bash
# rocprofv3 kernel trace + stats of the SL bench step.  Usage: scripts/profile_step.sh OUTDIR [bench args]
set -e
OUT=${1:-gpurun_out/prof}; shift || true
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -- python bench.py "$@"
