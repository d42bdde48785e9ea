#!/bin/bash
# Alternating A/B: bench.py without a process group vs the forced 1-rank RCCL process group
# (bucketed async all-reduce on RCCL inside the step), both under torch.distributed.run.
set -e
mkdir -p gpurun_out/rccl
export PYTHONPATH=$PWD
for rep in 1 2 3; do
  for f in 0 1; do
    ALPHAGO_AMD_FORCE_DIST=$f timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $((29540 + rep * 2 + f)) bench.py --gpus 1 --steps 40 --warmup 5 2>/dev/null \
      | grep metric | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('force_dist', $f, d['value'], d['ms_per_step'])" \
      | tee -a gpurun_out/rccl/ab.txt
  done
done
