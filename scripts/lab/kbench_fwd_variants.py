"""Forward-conv tile-variant sweep (3x3 192->192 and 5x5 64->192, B boards)."""
import argparse, json
import os, sys  # noqa: E401
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _lab import TILE, STAMPS, WGV, FP8V, FP8_OLD_TO_NEW, lab_conv_fwd, lab_conv_wgrad, lab_conv_fwd_fp8  # noqa: E402,F401
import torch
from alphago_amd import ops

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--tiles", default="0,128,256,2560,2568,384,32,2,-1")
a = ap.parse_args()
ops.load()
dev = torch.device("cuda")
B, F, S = a.batch, 192, 19
M = B * S * S
x = ops.padded_empty(B, S, 1, F, dev); x[:, 1:20, 1:20].normal_()
x0 = ops.padded_empty(B, S, 2, 64, dev); x0[:, 2:21, 2:21].normal_()
y = ops.padded_empty(B, S, 1, F, dev)
w = torch.randn(F, F, 3, 3, device=dev) * 0.05
w1 = torch.randn(F, 48, 5, 5, device=dev) * 0.05
wf = ops.packed_weight_like(w, F, F); wd = ops.packed_weight_like(w, F, F, True)
wf1 = ops.packed_weight_like(w1, 64, F)
ops.pack_weights([w, w1], [wf, wf1], [wd, torch.empty(0, device=dev, dtype=torch.bfloat16)])
bias = torch.zeros(F, device=dev)

def timeit(fn):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters * 1e3

fl3 = 2.0 * M * F * F * 9
fl5 = 2.0 * M * F * 64 * 25
ref = None
res = {}
for t in [int(s) for s in a.tiles.split(",")]:
    TILE[0] = t
    y.zero_()
    lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1)
    torch.cuda.synchronize()
    if ref is None: ref = y.clone()
    err = (y.float() - ref.float()).abs().max().item()
    t3 = timeit(lambda: lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1))
    t5 = timeit(lambda: lab_conv_fwd(x0, wf1, bias, y, 5, S, 2, 1))
    res[t] = dict(fwd3_us=round(t3, 1), fwd3_pf=round(fl3 / t3 / 1e9, 3), fwd5_us=round(t5, 1),
                  fwd5_pf=round(fl5 / t5 / 1e9, 3), maxdiff_vs_first=err)
    print(t, res[t], flush=True)
TILE[0] = 0
print(json.dumps(res))
