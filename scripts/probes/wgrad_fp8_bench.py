"""fp8 vs bf16 wgrad (+ reduce) of a value-net layer (160 -> 160 3x3), B = 1024, back to back."""
import json
import sys
import time

import torch

from alphago_amd import ops

ops.load()
dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
S, K, Cp = 19, 3, 160
M = B * S * S
x = ops.padded_empty(B, S, 1, Cp, dev)
x[:, 1:20, 1:20, :152].normal_()
dz = ops.padded_empty(B, S, 1, Cp, dev)
dz[:, 1:20, 1:20, :152].normal_()
x8 = torch.randint(0, 120, x.shape, dtype=torch.uint8, device=dev)
dz8 = torch.randint(0, 120, x.shape, dtype=torch.uint8, device=dev)
x8[:, 0] = 0
dz8[:, 0] = 0
gw = torch.zeros(152, 152, 3, 3, device=dev)
gb = torch.zeros(152, device=dev)
xs = torch.tensor([127], dtype=torch.int32, device=dev)
gm = torch.ones(1, device=dev)
ns16 = ops.wgrad_nsplit(M, Cp, Cp, K)
ns8 = ops.wgrad_fp8_nsplit(M)
s16 = torch.empty(ns16, 9, Cp, Cp, device=dev)
d16 = torch.zeros(ns16, Cp, device=dev)
s8 = torch.empty(ns8, 9, Cp, Cp, device=dev)
d8 = torch.zeros(ns8, Cp, device=dev)


def bf16():
    ops.conv_wgrad(x, dz, s16, d16, K, S, 1, 1)
    ops.conv_wgrad_reduce(s16, d16, gw, gb, 1.0, 0.0)


def fp8():
    ops.conv_wgrad_fp8(x8, dz8, s8, d8, xs, xs, gm, K, S, 1, 1)
    ops.conv_wgrad_reduce(s8, d8, gw, gb, 1.0, 0.0)


flops = 2.0 * M * 152 * 152 * 9
for rnd in range(2):
    for name, fn in (("bf16", bf16), ("fp8", fp8)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < secs:
            for _ in range(10):
                fn()
            n += 10
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"wgrad": name, "B": B, "us": round(dt / n * 1e6, 1), "pflops": round(n * flops / dt / 1e15, 3),
                          "nsplit": ns16 if name == "bf16" else ns8}), flush=True)
