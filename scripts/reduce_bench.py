"""Standalone timing of the deterministic split-K wgrad reduce (conv_wgrad_reduce) at the
SL-step shapes: 3x3 layer (56 splits x 9 taps x 192 x 192) and the 5x5 first layer
(102 splits x 25 taps x 192 x 64, 48 real input channels).  Prints us/call and the
effective slab read bandwidth."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from alphago_amd import ops

def run(ns, T, co, ci, ci_real, k):
    dev = torch.device("cuda")
    slab = torch.randn(ns, T, co, ci, device=dev)
    dbs = torch.randn(ns, co, device=dev)
    gw = torch.zeros(co, ci_real, k, k, device=dev)
    gb = torch.zeros(co, device=dev)
    for _ in range(5):
        ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    e0.record()
    for _ in range(n):
        ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    ref = slab[:, :, :, :ci_real].sum(0).permute(1, 2, 0).reshape(co, ci_real, k, k)
    err = (gw - ref).abs().max().item()
    print("ns=%d T=%d %dx%d: %.1f us/call, %.2f TB/s slab read, max err %.2e"
          % (ns, T, co, ci, us, slab.numel() * 4 / us / 1e6, err), flush=True)

run(56, 9, 192, 192, 192, 3)
run(102, 25, 192, 64, 48, 5)
