#!/bin/bash
# bench.py under several settings; each arg is "TILE:FLAGS" (TILE 0 = default)
export PYTHONPATH=$PWD
timeout -k 10 120 python bench.py --steps 10 --warmup 10 > /dev/null 2>&1  # warm the GPU
for v in "$@"; do
  t=${v%%:*}; f=${v#*:}; f=${f//,/ }
  if [ "$t" = "0" ]; then unset ALPHAGO_AMD_CONV_TILE; else export ALPHAGO_AMD_CONV_TILE=$t; fi
  timeout -k 10 240 python bench.py --steps 40 --warmup 20 $f 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])"
done
