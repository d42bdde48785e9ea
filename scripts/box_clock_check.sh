#!/bin/bash
# Box identity and sustained clocks/power during the SL bench (explains box-to-box spread)
set -e
O=gpurun_out/boxclk
mkdir -p $O
export PYTHONPATH=$PWD
amd-smi static -g 0 > $O/static.txt 2>&1 || true
( for i in $(seq 1 40); do amd-smi metric -g 0 2>&1 | grep -iE "GFX_0|GFX_CLK|SOCKET_POWER|POWER_LIMIT|CURRENT_SOCKET|THROTTLE|TEMP_HOTSPOT|HOTSPOT" | head -12; echo ---; sleep 1; done ) > $O/monitor.txt 2>&1 &
MON=$!
timeout -k 10 200 python3 bench.py --gpus 1 --steps 100 --warmup 5 > $O/bench.json 2> $O/bench.err
kill $MON 2>/dev/null || true
cut -c1-200 $O/bench.json
grep -iE "power_cap|POWER_LIMIT|max_power|SKU|MARKET|PRODUCT|PCIE|VBIOS" $O/static.txt | head -12 || true
