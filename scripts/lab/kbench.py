"""Per-kernel microbenchmark of the SL-step kernels at a given batch (standalone, no overlap)."""
import argparse, json
import os, sys  # noqa: E401
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _lab import TILE, STAMPS, WGV, FP8V, FP8_OLD_TO_NEW, lab_conv_fwd, lab_conv_wgrad, lab_conv_fwd_fp8  # noqa: E402,F401
import torch
from alphago_amd import ops

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--F", type=int, default=192)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--splits", default="")
a = ap.parse_args()
ops.load()
dev = torch.device("cuda")
B, F, S = a.batch, a.F, 19
M = B * S * S
x = ops.padded_empty(B, S, 1, F, dev); x[:, 1:20, 1:20].normal_()
x0 = ops.padded_empty(B, S, 2, 64, dev); x0[:, 2:21, 2:21].bernoulli_(torch.full_like(x0[:, 2:21, 2:21], 0.5, dtype=torch.float32).to(torch.bfloat16))
y = ops.padded_empty(B, S, 1, F, dev)
w = torch.randn(F, F, 3, 3, device=dev) * 0.05
w1 = torch.randn(F, 48, 5, 5, device=dev) * 0.05
wf = ops.packed_weight_like(w, F, F); wd = ops.packed_weight_like(w, F, F, True)
wf1 = ops.packed_weight_like(w1, 64, F)
ops.pack_weights([w, w1], [wf, wf1], [wd, torch.empty(0, device=dev, dtype=torch.bfloat16)])
bias = torch.zeros(F, device=dev)
gw = torch.zeros(F, F, 3, 3, device=dev); gb = torch.zeros(F, device=dev)

def timeit(fn):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters * 1e3  # us

res = {}
fl3 = 2.0 * M * F * F * 9
fl1 = 2.0 * M * F * 64 * 25
for bm in (256, 384):
    TILE[0] = bm
    for nm, fn in (("fwd3x3", lambda: lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1)),
                   ("dgrad3x3", lambda: lab_conv_fwd(x, wd, None, y, 3, S, 1, 1, mode=ops.MODE_MASK, mask=x)),
                   ("fwd5x5", lambda: lab_conv_fwd(x0, wf1, bias, y, 5, S, 2, 1))):
        k = "%s_bm%d" % (nm, bm)
        t = timeit(fn)
        res[k] = min(t, res.get(k, 1e30))
TILE[0] = 0
res["fwd3x3"] = timeit(lambda: lab_conv_fwd(x, wf, bias, y, 3, S, 1, 1))
res["fwd5x5"] = timeit(lambda: lab_conv_fwd(x0, wf1, bias, y, 5, S, 2, 1))
res["dgrad3x3"] = timeit(lambda: lab_conv_fwd(x, wd, None, y, 3, S, 1, 1, mode=ops.MODE_MASK, mask=x))
splits = [int(s) for s in a.splits.split(",")] if a.splits else [ops.wgrad_splits(M, 9)]
for ns in splits:
    slab = torch.empty(ns, 9, F, F, device=dev); dbs = torch.zeros(ns, F, device=dev)
    for rep in range(2):
        for v in (0, 2, 3):
            WGV[0] = v
            k = "wgrad3x3_v%d_s%d" % (v, ns)
            res[k] = min(res.get(k, 1e30), timeit(lambda: lab_conv_wgrad(x, y, slab, dbs, 3, S, 1, 1)))
    WGV[0] = 0
    res["reduce_s%d" % ns] = timeit(lambda: ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0))
# layer-0 wgrad (5x5, Cin 64): tap-merged (v0) vs one tap per workgroup (v1)
dz1 = y
for v, nss in ((1, (20,)), (0, (25, 51, 102))):
    WGV[0] = v
    for ns in nss:
        slab1 = torch.empty(ns, 25, F, 64, device=dev); dbs1 = torch.zeros(ns, F, device=dev)
        k = "wgrad5x5_v%d_s%d" % (v, ns)
        res[k] = min(res.get(k, 1e30), timeit(lambda: lab_conv_wgrad(x0, dz1, slab1, dbs1, 5, S, 2, 1)))
WGV[0] = 0
# fp8 forward (block-scaled MFMA), 3x3 and 5x5
x8 = torch.zeros(x.shape, dtype=torch.uint8, device=dev); ops.quantize_fp8(x, x8, 0)
x08 = torch.zeros(x0.shape, dtype=torch.uint8, device=dev); ops.quantize_fp8(x0, x08, 0)
w8, _ = ops.pack_weights_fp8(w, F, F); w18, _ = ops.pack_weights_fp8(w1, F, 64)
sc = torch.tensor([127, 127], dtype=torch.int32, device=dev); osc = torch.ones(1, device=dev)
y8 = torch.zeros(y.shape, dtype=torch.uint8, device=dev)
res["fp8_fwd3x3"] = timeit(lambda: lab_conv_fwd_fp8(x8, w8, bias, sc, osc, 3, S, 1, 1, y_fp8=y8))
am = ops.fp8_amax_buffer(1, dev)[0]
res["fp8_fwd3x3_amax"] = timeit(lambda: lab_conv_fwd_fp8(x8, w8, bias, sc, osc, 3, S, 1, 1, y_fp8=y8, amax=am))
res["fp8_fwd3x3_dual"] = timeit(lambda: lab_conv_fwd_fp8(x8, w8, bias, sc, osc, 3, S, 1, 1, y_fp8=y8, y_bf16=y, amax=am))
res["fp8_fwd5x5"] = timeit(lambda: lab_conv_fwd_fp8(x08, w18, bias, sc, osc, 5, S, 2, 1, y_fp8=y8))
# fused policy head (train) on the last activation
hw = torch.randn(F, device=dev) * 0.05; hb = torch.zeros(1, device=dev)
tgt = torch.randint(0, 361, (B,), dtype=torch.int32, device=dev)
dz = ops.padded_empty(B, S, 1, F, dev); lo = torch.zeros(B, device=dev); co = torch.zeros(B, device=dev)
dh = torch.zeros(B, F + 1, device=dev)
res["policy_head_train"] = timeit(lambda: ops.policy_head_train(x, hw, hb, tgt, dz, lo, co, dh, S, 1.0 / B))
out = {k: {"us": round(v, 1), "TF": round((fl1 if "5x5" in k else fl3) / (v * 1e-6) / 1e12, 1) if "reduce" not in k else None} for k, v in res.items()}
print(json.dumps({"batch": B, "F": F, **out}))
