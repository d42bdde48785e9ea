"""Run one kernel many times (for PMC collection): fwd | dgrad | wgrad."""
import sys, torch
import os, sys  # noqa: E401
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _lab import TILE, STAMPS, WGV, FP8V, FP8_OLD_TO_NEW, lab_conv_fwd, lab_conv_wgrad, lab_conv_fwd_fp8  # noqa: E402,F401
from alphago_amd import ops
ops.load()
which = sys.argv[1]; B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
import os
if which.endswith("ring"):  # forward/dgrad on the ring-pipelined tiling
    TILE[0] = 32
    which = which[:-4]
if os.environ.get("ALPHAGO_AMD_CONV_TILE"):
    TILE[0] = int(os.environ["ALPHAGO_AMD_CONV_TILE"])
dev = torch.device("cuda"); S, F = 19, 192; M = B * S * S
x = ops.padded_empty(B, S, 1, F, dev); x[:, 1:20, 1:20].normal_()
y = ops.padded_empty(B, S, 1, F, dev)
w = torch.randn(F, F, 3, 3, device=dev) * 0.05
wf = ops.packed_weight_like(w, F, F); wd = ops.packed_weight_like(w, F, F, True)
ops.pack_weights([w], [wf], [wd])
bias = torch.zeros(F, device=dev)
ns = ops.wgrad_splits(M, 9)
slab = torch.empty(ns, 9, F, F, device=dev); dbs = torch.zeros(ns, F, device=dev)
if which == "fp8":
    x8 = torch.zeros(x.shape, dtype=torch.uint8, device=dev); ops.quantize_fp8(x, x8, 0)
    w8, _ = ops.pack_weights_fp8(w, F, F)
    y8 = torch.zeros(x.shape, dtype=torch.uint8, device=dev)
    sc = torch.tensor([127, 127], dtype=torch.int32, device=dev); osc = torch.ones(1, device=dev)
for _ in range(10):
    if which == "fp8": lab_conv_fwd_fp8(x8, w8, bias, sc, osc, 3, S, 1, 1, y_fp8=y8)
    elif which == "fwd": lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1)
    elif which == "dgrad": lab_conv_fwd(x, wd, None, y, 3, S, 1, 1, mode=ops.MODE_MASK, mask=x)
    else: lab_conv_wgrad(x, y, slab, dbs, 3, S, 1, 1)
torch.cuda.synchronize()
