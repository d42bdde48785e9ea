#!/bin/bash
# Power-limited steady-state A/B of conv kernels (10 s each, socket power sampled by amd-smi).
# KERNELS="fwd:385 fwd:386 fwd:lab5 ..." (see scripts/probes/conv_power_probe.py)
set -e
O=${OUT:-gpurun_out/cpab}
mkdir -p $O
export PYTHONPATH=$PWD
for k in ${KERNELS:-fwd:385 fwd:386 fwd:lab5 dgrad:385 dgrad:386 dgrad:lab5}; do
  ( for i in $(seq 1 14); do amd-smi metric -g 0 2>&1 | grep -E "SOCKET_POWER:" | head -1; sleep 0.6; done ) > $O/power_${k/:/_}.txt 2>&1 &
  MON=$!
  timeout -k 10 90 python scripts/probes/conv_power_probe.py $k ${SECS:-10} | tee -a $O/result.txt
  kill $MON 2>/dev/null || true
  wait $MON 2>/dev/null || true
  echo "$k power: $(grep -o '[0-9]* W' $O/power_${k/:/_}.txt | tr '\n' ' ')" | tee -a $O/result.txt
done
