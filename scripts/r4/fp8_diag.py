"""Round-4 diagnosis of the fp8 value trainer at width 152 (padded 160): which stage separates the HIP
fp8 step from the exact fp32 autograd of the same quantised forward?  Arms: (fp8_dgrad, fp8_wgrad) in
FF / TF / FT / TT on the 12 x 152 value net; per arm the max |value| difference of the forward, the
head-parameter gradient cosines (forward only) and every trunk layer's weight-gradient cosine / norm
ratio.  Usage: python scripts/r4/fp8_diag.py [--batch 64] [--planes random|games]"""
import argparse
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def emulate(net, planes, z, wscale, osc):
    def ste(x, q):
        return x + (q - x).detach()

    h = planes.float()
    L = len(net.trunk.weights)
    for l, (w, b, k) in enumerate(zip(net.trunk.weights, net.trunk.biases, net.trunk.widths)):
        s = float(wscale[l])
        wq = ste(w, (w.detach() * s).clamp(-448, 448).to(torch.float8_e4m3fn).float() / s)
        y = F.relu(F.conv2d(h, wq, b, padding=k // 2))
        if l < L - 1:
            o = float(osc[l])
            h = ste(y, (y.detach() * o).clamp(max=448).to(torch.float8_e4m3fn).float() / o)
        else:
            h = ste(y, y.detach().bfloat16().float())
    zz = F.conv2d(h, net.head_w, net.head_b).flatten(1)
    v = torch.tanh((zz @ net.fc1_w + net.fc1_b) @ net.fc2_w + net.fc2_b).squeeze(1)
    loss = ((v - z) ** 2).sum() / len(z)
    params = dict(net.named_parameters())
    g = torch.autograd.grad(loss, list(params.values()))
    return v.detach(), dict(zip(params.keys(), g))


def ref_name(name):
    """trainer flat-parameter name -> ValueNet parameter name"""
    if name[0] in "wb" and name[1:].isdigit():
        return "trunk.%s.%s" % ("weights" if name[0] == "w" else "biases", name[1:])
    return name


def main():
    from alphago_amd.models.nets import ValueNet
    from alphago_amd.train.engine import HipValueTrainer

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--planes", default="random")
    ap.add_argument("--layers", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = a.batch
    if a.planes == "random":
        g = torch.Generator().manual_seed(11)
        planes = torch.randint(0, 2, (B, 49, 19, 19), dtype=torch.uint8, generator=g)
    else:
        from alphago_amd.data.synthetic import random_game_states
        from alphago_amd.features import VALUE_FEATURES, Preprocess
        planes = torch.from_numpy(Preprocess(VALUE_FEATURES).states_to_uint8(
            random_game_states(B, np.random.default_rng(0))))
    planes = planes.to(dev)
    torch.manual_seed(4)
    z = torch.rand(B, device=dev) * 2 - 1
    net0 = ValueNet(49, filters_per_layer=152, layers=a.layers)
    for dg, wg in [(False, False), (True, False), (False, True), (True, True)]:
        net = copy.deepcopy(net0)
        ref = copy.deepcopy(net0).to(dev)
        t8 = HipValueTrainer(net, B, lr=0.0, device=dev, precision="fp8", fp8_dgrad=dg, fp8_wgrad=wg)
        t8.compute_grads(planes, z)
        osc, wscale = t8.osc8.clone(), t8.wscale8.clone()
        t8.compute_grads(planes, z)
        torch.cuda.synchronize()
        v_ref, g_ref = emulate(ref, planes, z, wscale.cpu(), osc.cpu())
        out = {"fp8_dgrad": dg, "fp8_wgrad": wg, "flags": [t8.fp8_dgrad, t8.fp8_wgrad],
               "value_maxdiff": round(float((t8.val - v_ref).abs().max()), 5),
               "value_absmax": round(float(v_ref.abs().max()), 4)}
        cos = {}
        for name in t8.fp.names:
            ga = t8.fp.grad_views[name].double().flatten()
            gb = g_ref[ref_name(name)]
            gb = gb.double().flatten()
            cos[name] = (round(float(F.cosine_similarity(ga, gb, dim=0)), 4), round(float(ga.norm() / gb.norm()), 4))
        out["grads"] = cos
        print(json.dumps(out), flush=True)
        del t8
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
