"""CPU emulation of the fp8 value-training numerics (which quantisation scheme keeps the 12-layer trunk's
weight gradients close to fp32?).  Runs on the CPU with torch's float8 dtypes; the GPU kernels
implement the chosen scheme (conv_fp8.hip, conv_wgrad_fp8.hip).

Each conv layer's forward multiplies e4m3 weights by e4m3 activations; its backward quantises the
output gradient dZ once and uses it for both the dgrad (dZ x e4m3 weights) and the wgrad (dZ x the
forward's e4m3 input), as the all-fp8 HIP backward does.  Schemes:
  grad format  e5m2 (round 3) | e4m3
  grad scale   tensor (one power of two per tensor) | block (one per 32 channels of a pixel, the
               MFMA's per-lane E8M0 block scale along the dgrad's K)
  act scale    tensor | block
Reports per-parameter cosine vs the fp32 gradient, at random init and after N SGD steps on the
value-teacher task (data/synthetic.py).

Usage: python scripts/fp8_grad_sim.py [--batch 32] [--train-steps 40] [--filters 152] [--layers 12]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

E4M3_MAX, E5M2_MAX = 448.0, 57344.0


def q_tensor(x, fmt):
    """Per-tensor power-of-two scale (largest element just below the format's max), round to fmt."""
    mx = E4M3_MAX if fmt == "e4m3" else E5M2_MAX
    dt = torch.float8_e4m3fn if fmt == "e4m3" else torch.float8_e5m2
    amax = x.abs().max().clamp_min(1e-30)
    e = torch.floor(torch.log2(mx / amax))
    s = torch.pow(2.0, e)
    return (x * s).clamp(-mx, mx).to(dt).float() / s


def q_block(x, fmt, block=32):
    """Power-of-two scale per 32 consecutive channels of each pixel (NCHW: channel axis 1)."""
    mx = E4M3_MAX if fmt == "e4m3" else E5M2_MAX
    dt = torch.float8_e4m3fn if fmt == "e4m3" else torch.float8_e5m2
    B, C, H, W = x.shape
    pad = (-C) % block
    xp = F.pad(x, (0, 0, 0, 0, 0, pad)) if pad else x
    xb = xp.view(B, (C + pad) // block, block, H, W)
    amax = xb.abs().amax(2, keepdim=True).clamp_min(1e-30)
    s = torch.pow(2.0, torch.floor(torch.log2(mx / amax)))
    y = ((xb * s).clamp(-mx, mx).to(dt).float() / s).view(B, C + pad, H, W)
    return y[:, :C] if pad else y


class QConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, cfg):
        fq = not cfg["fp32"] and cfg.get("fwd", True)
        if fq and cfg.get("bf16"):
            xq, wq = x.bfloat16().float(), w.bfloat16().float()
        else:
            qa, qw = fq and cfg.get("acts", True), fq and cfg.get("weights", True)
            xq = x if not qa else (q_block(x, "e4m3") if cfg["act"] == "block" else q_tensor(x, "e4m3"))
            wq = w if not qw else q_tensor(w, "e4m3")
        y = F.conv2d(xq, wq, b, padding=w.shape[2] // 2)
        ctx.save_for_backward(xq, wq)
        ctx.cfg = cfg
        ctx.pad = w.shape[2] // 2
        return y

    @staticmethod
    def backward(ctx, gy):
        xq, wq = ctx.saved_tensors
        cfg = ctx.cfg
        if not cfg["fp32"] and cfg["gfmt"] is not None:
            gy = q_block(gy, cfg["gfmt"]) if cfg["gscale"] == "block" else q_tensor(gy, cfg["gfmt"])
        gx = torch.nn.grad.conv2d_input(xq.shape, wq, gy, padding=ctx.pad)
        gw = torch.nn.grad.conv2d_weight(xq, wq.shape, gy, padding=ctx.pad)
        return gx, gw, gy.sum((0, 2, 3)), None


def forward(net, x, cfg):
    h = x
    L = len(net.trunk.weights)
    keep = set(l % L for l in cfg.get("bf16_layers", ()))
    for l, (w, b) in enumerate(zip(net.trunk.weights, net.trunk.biases)):
        h = F.relu(QConv.apply(h, w, b, dict(cfg, bf16=True) if l in keep else cfg))
    z = F.conv2d(h, net.head_w, net.head_b).flatten(1)
    z = z @ net.fc1_w + net.fc1_b
    return torch.tanh(z @ net.fc2_w + net.fc2_b).squeeze(1)


def grads(net, x, z, cfg):
    net.zero_grad()
    v = forward(net, x, cfg)
    ((v - z) ** 2).sum().div(len(z)).backward()
    return {n: p.grad.detach().clone() for n, p in net.named_parameters()}


def main():
    from alphago_amd.data.synthetic import random_game_states, value_teacher, value_teacher_pool
    from alphago_amd.features import VALUE_FEATURES, Preprocess
    from alphago_amd.models.nets import ValueNet

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--train-steps", type=int, default=40)
    ap.add_argument("--filters", type=int, default=152)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--lr", type=float, default=0.02)
    a = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    rng = np.random.default_rng(0)
    probe = Preprocess(VALUE_FEATURES).states_to_uint8(random_game_states(256, rng))
    teacher = value_teacher(49, a.filters, a.layers, probe=probe)
    n = a.batch * (a.train_steps + 1)
    planes, tz = value_teacher_pool(n, teacher, seed=1, symmetrize=False)
    X = torch.from_numpy(planes).float()
    Z = torch.from_numpy(tz).float()
    torch.manual_seed(5)
    net = ValueNet(49, filters_per_layer=a.filters, layers=a.layers)
    schemes = {
        "e5m2/tensor grads, tensor acts (round 3)": dict(gfmt="e5m2", gscale="tensor", act="tensor"),
        "e4m3/tensor grads, tensor acts": dict(gfmt="e4m3", gscale="tensor", act="tensor"),
        "e5m2/block grads, block acts": dict(gfmt="e5m2", gscale="block", act="block"),
        "e4m3/block grads, block acts": dict(gfmt="e4m3", gscale="block", act="block"),
        "fp8 forward only (exact backward of the quantised net)": dict(gfmt=None, gscale="tensor", act="tensor"),
        "e4m3 weights only": dict(gfmt=None, gscale="tensor", act="tensor", acts=False),
        "e4m3 activations only": dict(gfmt=None, gscale="tensor", act="tensor", weights=False),
        "bf16 forward (weights + activations), fp32 backward": dict(gfmt=None, gscale="tensor", act="tensor", bf16=True),
        "e4m3 forward, first layer bf16": dict(gfmt=None, gscale="tensor", act="tensor", bf16_layers=(0,)),
        "e4m3 forward, last layer bf16": dict(gfmt=None, gscale="tensor", act="tensor", bf16_layers=(-1,)),
        "e4m3 forward, first + last layers bf16": dict(gfmt=None, gscale="tensor", act="tensor", bf16_layers=(0, -1)),
        "e5m2 tensor grads only (fp32 forward)": dict(gfmt="e5m2", gscale="tensor", act="tensor", fwd=False),
        "e4m3 block grads only (fp32 forward)": dict(gfmt="e4m3", gscale="block", act="block", fwd=False),
    }
    out = {}

    def report(tag):
        xb, zb = X[:a.batch], Z[:a.batch]
        ref = grads(net, xb, zb, dict(fp32=True))
        res = {}
        for name, sc in schemes.items():
            g = grads(net, xb, zb, dict(fp32=False, **sc))
            cos = {k: round(float(F.cosine_similarity(g[k].flatten().double(), ref[k].flatten().double(), dim=0)), 4)
                   for k in ref if k.startswith("trunk.weights")}
            res[name] = {"min": min(cos.values()), "mean": round(float(np.mean(list(cos.values()))), 4),
                         "per_layer": [cos["trunk.weights.%d" % l] for l in range(a.layers)]}
            print(tag, name, res[name]["min"], res[name]["mean"], flush=True)
        out[tag] = res

    report("init")
    opt = torch.optim.SGD(net.parameters(), lr=a.lr)
    for s in range(1, a.train_steps + 1):
        xb, zb = X[s * a.batch:(s + 1) * a.batch], Z[s * a.batch:(s + 1) * a.batch]
        opt.zero_grad()
        ((forward(net, xb, dict(fp32=True)) - zb) ** 2).mean().backward()
        opt.step()
    report("after_%d_steps" % a.train_steps)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
