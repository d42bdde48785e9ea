#!/bin/bash
# Round 4 batch GD: per-genmove diagnosis (evaluations, overflow fallbacks, host time split).
O=gpurun_out/r4_gd${GDTAG:-}
mkdir -p $O
export PYTHONPATH=$PWD
source scripts/r4/lib.sh
step diag 240 python3 -u scripts/r4/genmove_diag.py
