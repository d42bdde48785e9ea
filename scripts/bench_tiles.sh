#!/bin/bash
# bench.py under several forward/dgrad tile settings (ALPHAGO_AMD_CONV_TILE); one line each
export PYTHONPATH=$PWD
for t in ${@:-0 9 10}; do
  if [ "$t" = "0" ]; then unset ALPHAGO_AMD_CONV_TILE; else export ALPHAGO_AMD_CONV_TILE=$t; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('tile', '$t', d['value'], d['ms_per_step'])"
done
