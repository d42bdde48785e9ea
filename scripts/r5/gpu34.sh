#!/bin/bash
O=gpurun_out/r5/b34
mkdir -p $O
export PYTHONPATH=$PWD PYTHONUNBUFFERED=1 TMPDIR=/tmp
source scripts/r5/lib.sh
step fp8 300 python -u scripts/r5/fp8_sl_diag.py fp8
grep step $O/fp8.log | cut -c1-400
step fp8sr 300 env ALPHAGO_AMD_FP8_SR=1 python -u scripts/r5/fp8_sl_diag.py fp8
grep step $O/fp8sr.log | cut -c1-200
step bf16 300 python -u scripts/r5/fp8_sl_diag.py bf16
grep step $O/bf16.log | cut -c1-200
