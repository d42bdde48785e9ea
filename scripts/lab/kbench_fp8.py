"""fp8 forward conv: LDS-staged (variant 0) vs pixel operand from L2 (variant 1),
3x3 192->192 and 5x5 64->192 at batch B (default 1024), random operands."""
import argparse, json
import os, sys  # noqa: E401
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _lab import TILE, STAMPS, WGV, FP8V, FP8_OLD_TO_NEW, lab_conv_fwd, lab_conv_wgrad, lab_conv_fwd_fp8  # noqa: E402,F401
import torch
from alphago_amd import ops

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--variants", default="0,1,0,1")
a = ap.parse_args()
ops.load()
dev = torch.device("cuda")
B, F, S = a.batch, 192, 19
M = B * S * S
x = ops.padded_empty(B, S, 1, F, dev); x[:, 1:20, 1:20].normal_()
x0 = ops.padded_empty(B, S, 2, 64, dev); x0[:, 2:21, 2:21].normal_()
w = torch.randn(F, F, 3, 3, device=dev) * 0.05
w1 = torch.randn(F, 64, 5, 5, device=dev) * 0.05
bias = torch.zeros(F, device=dev)
x8 = torch.zeros(x.shape, dtype=torch.uint8, device=dev); ops.quantize_fp8(x, x8, 0)
x08 = torch.zeros(x0.shape, dtype=torch.uint8, device=dev); ops.quantize_fp8(x0, x08, 0)
w8, _ = ops.pack_weights_fp8(w, F, F); w18, _ = ops.pack_weights_fp8(w1, F, 64)
sc = torch.tensor([127, 127], dtype=torch.int32, device=dev); osc = torch.ones(1, device=dev)
y8 = torch.zeros((B, S + 2, S + 2, F), dtype=torch.uint8, device=dev)
yb = ops.padded_empty(B, S, 1, F, dev)


def timeit(fn):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters * 1e3


fl3, fl5 = 2.0 * M * F * F * 9, 2.0 * M * F * 64 * 25
ref = None
out = {}
for v in [int(t) for t in a.variants.split(",")]:
    FP8V[0] = FP8_OLD_TO_NEW[v]
    yb.zero_()
    lab_conv_fwd_fp8(x8, w8, bias, sc, osc, 3, S, 1, 1, y_bf16=yb)
    torch.cuda.synchronize()
    if ref is None:
        ref = yb.float().clone()
    d = float((yb.float() - ref).abs().max())
    t3 = timeit(lambda: lab_conv_fwd_fp8(x8, w8, bias, sc, osc, 3, S, 1, 1, y_fp8=y8))
    t5 = timeit(lambda: lab_conv_fwd_fp8(x08, w18, bias, sc, osc, 5, S, 2, 1, y_fp8=y8))
    r = {"fwd3_us": round(t3, 1), "fwd3_pf": round(fl3 / t3 / 1e9, 3), "fwd5_us": round(t5, 1),
         "fwd5_pf": round(fl5 / t5 / 1e9, 3), "maxdiff_vs_first": d}
    print(v, r, flush=True)
    out[str(v)] = r
FP8V[0] = FP8_OLD_TO_NEW[2]
print(json.dumps(out))
