#!/bin/bash
# Rehearsal of the driver's multi-GPU bench form on the 1-GPU box: two HIP ranks on cuda:0 under
# torch.distributed.run with the gloo backend (RCCL refuses two ranks on one device,
# profiles/r2_rccl_same_gpu.md) -- the rows gather, bucketed all-reduce and max-over-ranks timing.
O=gpurun_out/r6/dp2
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
export ALPHAGO_AMD_DIST_BACKEND=gloo
step dp2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --min-warmup-s 0 --batch 512
grep -h '"value"' $O/dp2.log | cut -c1-400
