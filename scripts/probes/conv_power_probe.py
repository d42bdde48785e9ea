"""One conv kernel of the SL step run back to back for ~10 s at B = 2176 (the power-limited steady
state); the caller samples socket power.  Usage: conv_power_probe.py KIND:TILE [secs]
  KIND  fwd (3x3, 192 -> 192, bias + ReLU + bitmask), dgrad (3x3, bitmask ReLU'), fwd5 (5x5 layer 0,
        48 planes padded to 64), wgrad (3x3 split-K + reduce), wino (kernel-lab Winograd forward,
        bias + ReLU, PF counted as the direct conv's FLOPs)
  TILE  a production tile code (0, 384-387) or labN for a kernel-lab tiling"""
import json
import sys
import time

import torch
from alphago_amd import ops

ops.load()
dev = torch.device("cuda")
kind, tile = sys.argv[1].split(":")
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
B, S, F = 2176, 19, 192
M = B * S * S
torch.manual_seed(0)
x = ops.padded_empty(B, S, 1, F, dev)
x[:, 1:20, 1:20].normal_()
x0 = ops.padded_empty(B, S, 2, 64, dev)
x0[:, 2:21, 2:21, :48].bernoulli_(torch.full_like(x0[:, 2:21, 2:21, :48], 0.5, dtype=torch.float32).bfloat16())
w = torch.randn(F, F, 3, 3, device=dev) * 0.05
w1 = torch.randn(F, 48, 5, 5, device=dev) * 0.05
wf, wd = ops.packed_weight_like(w, F, F), ops.packed_weight_like(w, F, F, True)
wf1 = ops.packed_weight_like(w1, 64, F)
ops.pack_weights([w, w1], [wf, wf1], [wd, torch.empty(0, device=dev, dtype=torch.bfloat16)])
bias = torch.randn(F, device=dev) * 0.1
y = ops.padded_empty(B, S, 1, F, dev)
mb = torch.zeros((B * (S + 2) ** 2 * ops.mbits_words(F),), dtype=torch.int32, device=dev)
ops.conv_fwd(x, wf, bias, y, 3, S, 1, 1, mbits=mb)  # ReLU' bits for the dgrad
L = None
if tile.startswith("lab"):
    L = ops.lab()
    code = int(tile[3:])
else:
    code = int(tile)


def fwd(xx, ww, K, P, mode=0, bits=None, out=y, b=bias):
    if L is None:
        ops.conv_fwd(xx, ww, b, out, K, S, P, 1, mode=mode, mbits=bits, tile=code)
    else:
        L.conv_fwd(xx, ww, b, None, out, K, S, P, 1, mode, bits, code, None)


dx = ops.padded_empty(B, S, 1, F, dev)
if kind == "fwd":
    fn, flops = (lambda: fwd(x, wf, 3, 1, bits=mb)), 2.0 * M * F * F * 9
elif kind == "dgrad":
    fn, flops = (lambda: fwd(y, wd, 3, 1, mode=ops.MODE_MASKBITS, bits=mb, out=dx, b=None)), 2.0 * M * F * F * 9
elif kind == "wino":  # kernel-lab Winograd F(2x2,3x3) forward (bias + ReLU); direct-equivalent FLOPs
    WL = ops.lab()
    u = ops.wino_pack_weights(w)
    fn, flops = (lambda: WL.wino_fwd(x, u, bias, y, S)), 2.0 * M * F * F * 9
elif kind == "fwd5":
    fn, flops = (lambda: fwd(x0, wf1, 5, 2)), 2.0 * M * F * 48 * 25
elif kind == "wgrad":
    # one resident round of the chosen kernel (production: per-tap, 0; lab5 = the row kernel)
    ns = ops.wgrad_nsplit(M, F, F, 3, variant=code)
    slab = torch.empty(ns, 9, F, F, device=dev)
    dbs = torch.zeros(ns, F, device=dev)
    gw = torch.zeros(F, F, 3, 3, device=dev)
    gb = torch.zeros(F, device=dev)

    def fn():
        if L is None:
            ops.conv_wgrad(x, y, slab, dbs, 3, S, 1, 1, variant=code)  # 0 per-tap, 6 tap pairs, 5 rows
        else:
            L.conv_wgrad(x, y, slab, dbs, 3, S, 1, 1, 0, code)  # lab5: row kernel
        ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    flops = 2.0 * M * F * F * 9
else:
    raise SystemExit("unknown kind " + kind)

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
print(json.dumps({"kernel": sys.argv[1], "us": round(dt / n * 1e6, 1), "pflops": round(n * flops / dt / 1e15, 3)}),
      flush=True)
