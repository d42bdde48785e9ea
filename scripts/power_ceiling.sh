#!/bin/bash
# bf16 throughput at the 1400 W socket limit: hipBLASLt GEMM vs the direct conv, with power samples
set -e
O=gpurun_out/pwr
mkdir -p $O
export PYTHONPATH=$PWD
for k in ${KERNELS:-gemm conv gemm conv}; do
  ( for i in $(seq 1 12); do amd-smi metric -g 0 2>&1 | grep -E "SOCKET_POWER:" | head -1; sleep 0.5; done ) > $O/power_$k.txt 2>&1 &
  MON=$!
  timeout -k 10 60 python scripts/probes/power_ceiling_probe.py $k | tee -a $O/result.txt
  kill $MON 2>/dev/null || true
  wait $MON 2>/dev/null || true
  echo "$k power samples: $(grep -o '[0-9]* W' $O/power_$k.txt | tr '\n' ' ')" | tee -a $O/result.txt
done
