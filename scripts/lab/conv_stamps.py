"""Per-segment cycle stamps of the ping-pong forward conv kernels (diagnostic build path).
usage: conv_stamps.py TILE   (4 = gather ping-pong, 5 = halo ping-pong)"""
import sys
import os, sys  # noqa: E401
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _lab import TILE, STAMPS, WGV, FP8V, FP8_OLD_TO_NEW, lab_conv_fwd, lab_conv_wgrad, lab_conv_fwd_fp8  # noqa: E402,F401
import torch
from alphago_amd import ops
ops.load()
tile = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda")
B, F, S = 1024, 192, 19
x = ops.padded_empty(B, S, 1, F, dev); x[:, 1:20, 1:20].normal_()
y = ops.padded_empty(B, S, 1, F, dev)
w = torch.randn(F, F, 3, 3, device=dev) * 0.05
wf = ops.packed_weight_like(w, F, F)
ops.pack_weights([w], [wf])
bias = torch.zeros(F, device=dev)
M = B * S * S
nwg = (M + 255) // 256
dbg = torch.zeros(nwg * 8 * 8, dtype=torch.int64, device=dev)
TILE[0] = tile
for _ in range(3):
    lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1)
STAMPS[0] = dbg
for _ in range(3):
    lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1)
torch.cuda.synchronize()
STAMPS[0] = None
d = dbg.view(nwg, 8, 8).double().cpu()
nk = 27 if tile != 6 else 27
names = ["ds_read issue", "glds/halo/ep issue", "lgkmcnt(0)", "barrier1", "mfma issue", "vmcnt (grp0 W)", "barrier2"]
for g in (0, 1):
    sub = d[:, 4 * g:4 * g + 4]
    print("group %d: wave lifetime %.0f cycles, %.0f per step" % (g, sub[..., 7].mean(), sub[..., 7].mean() / nk))
    for i, n in enumerate(names):
        print("   %-20s %8.1f cycles/step" % (n, sub[..., i].mean() / nk))
