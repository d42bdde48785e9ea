"""Segment-cycle stamps of the ping-pong forward conv (diagnostic build path)."""
import os, sys  # noqa: E401
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _lab import TILE, STAMPS, WGV, FP8V, FP8_OLD_TO_NEW, lab_conv_fwd, lab_conv_wgrad, lab_conv_fwd_fp8  # noqa: E402,F401
import torch
from alphago_amd import ops
ops.load()
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
TILE[0] = 4
for _ in range(3):
    lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1)
STAMPS[0] = dbg
for _ in range(3):
    lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1)
torch.cuda.synchronize()
STAMPS[0] = None
d = dbg.view(nwg, 8, 8).double().cpu()
raw = dbg.view(nwg, 8, 8)[..., 7].cpu()
nk = float(raw[0, 0] & 0xFFFF)
dsr = (raw >> 16).double()
names = ["ds_read+glds issue", "retire vmcnt", "lgkmcnt(0)", "barrier1", "mfma issue", "barrier2"]
for g in (0, 1):
    sub = d[:, 4 * g:4 * g + 4]
    print("group %d: wave lifetime %.0f cycles, %.0f per phase (nK=%d)" % (g, sub[..., 6].mean(), sub[..., 6].mean() / nk, nk))
    print("   %-20s %8.1f cycles/phase" % ("(ds_read issue part)", dsr[:, 4 * g:4 * g + 4].mean() / nk))
    for i, n in enumerate(names):
        print("   %-20s %8.1f cycles/phase" % (n, sub[..., i].mean() / nk))
