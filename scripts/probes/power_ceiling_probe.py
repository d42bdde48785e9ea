"""Throughput at the socket power limit: hipBLASLt bf16 GEMM vs our direct 3x3 conv, each run for
~10 s (long enough for the power controller to settle); power is sampled by the caller."""
import json
import sys
import time

import torch
from alphago_amd import ops

ops.load()
dev = torch.device("cuda")
which = sys.argv[1]


def run_for(fn, flops, secs=10.0):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < secs:
        for _ in range(20):
            fn()
        n += 20
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return n * flops / dt / 1e15


if which == "gemm":
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    c = torch.empty(8192, 8192, device=dev, dtype=torch.bfloat16)
    pf = run_for(lambda: torch.matmul(a, b, out=c), 2 * 8192 ** 3)
else:
    B, S, F = 2176, 19, 192
    x = ops.padded_empty(B, S, 1, F, dev)
    x[:, 1:20, 1:20].normal_()
    w = torch.randn(F, F, 3, 3, device=dev) * 0.05
    wf = ops.packed_weight_like(w, F, F)
    ops.pack_weights([w], [wf])
    bias = torch.zeros(F, device=dev)
    y = ops.padded_empty(B, S, 1, F, dev)
    flops = 2 * B * S * S * F * F * 9
    if which == "conv":
        pf = run_for(lambda: ops.conv_fwd(x, wf, bias, y, 3, S, 1, 1), flops)
    else:  # kernel-lab tilings, e.g. lab5 = compact halo + ping-pong, lab2 = interior halo
        tile = int(which[3:])
        L = ops.lab()
        pf = run_for(lambda: L.conv_fwd(x, wf, bias, None, y, 3, S, 1, 1, 0, None, tile, None), flops)
print(json.dumps({"kernel": which, "pflops": round(pf, 3)}), flush=True)
