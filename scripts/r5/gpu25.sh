#!/bin/bash
O=gpurun_out/r5/b25
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step cprof16 300 python -u scripts/r5/step_cprofile.py 16
head -60 $O/cprof16.log | tail -45
