"""Value-network precision parity on a learnable task (BASELINE config 5: value-net training on the fp8
MFMA conv path; reference value net AlphaGo/models/value.py:12-31, MSE on a tanh output).

Task (alphago_amd/data/synthetic.py value_teacher_pool): random-game positions in the value net's 49
planes, each labelled with a fixed random-init value teacher's tanh output (12 x 152, last layer
rescaled so its outputs spread over (-1, 1)), averaged over the 8 board symmetries.  A student of the
same architecture trains on it with per-sample random D4 augmentation; the held-out MSE per epoch is
the quality figure.

Arms (same data, same student initialisation, same batch order and symmetries):
  torch-fp32  the autograd trainer in fp32 (numerics oracle)
  hip-bf16    the HIP trainer, bf16 convs
  hip-fp8     the HIP trainer, fp8 conv path (e4m3 forward, e5m2 x e4m3 dgrad / wgrad: the default)
  hip-fp8fwd  the HIP trainer, e4m3 forward and bf16 backward (where the fp8 loss comes from)
  hip-fp8sr   hip-fp8 with stochastic rounding of the forward's e4m3 activations (ALPHAGO_AMD_FP8_SR)
  hip-fp8mix  per-layer precision: the --bf16-layers (default the first and last trunk layers) in bf16,
              the rest all-fp8; hip-fp8mixsr adds the stochastic rounding
After the first epoch the script also compares one batch's gradients of the fp8 and the fp32 trainer
at the bf16 arm's weights (per-layer cosine), on the 12-layer trunk.

Usage: python scripts/value_fp8_parity.py OUT_JSON [--positions N] [--epochs E] [--arms a,b,c]
       [--task teacher|material] [--init keras|he] [--lr R] [--optimizer sgd|momentum|adam] [--seeds N]
Prints one JSON line and writes it to OUT_JSON."""
import argparse
import copy
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alphago_amd.data.synthetic import random_game_states, value_teacher, value_teacher_pool  # noqa: E402
from alphago_amd.features import VALUE_FEATURES, Preprocess  # noqa: E402
from alphago_amd.models.nets import ValueNet  # noqa: E402
from alphago_amd.train.engine import HipValueTrainer, TorchValueTrainer  # noqa: E402


OPT = {}  # optimizer keywords of every arm (--optimizer / --momentum)
BF16_LAYERS = ()  # --bf16-layers: the layers the hip-fp8mix arms keep in bf16


def make_trainer(arm, net, B, lr, dev):
    if arm == "torch-fp32":
        return TorchValueTrainer(net, B, lr=lr, device=dev, **OPT)
    if arm == "hip-fp8fwd":  # e4m3 forward, bf16 backward
        return HipValueTrainer(net, B, lr=lr, device=dev, precision="fp8", fp8_dgrad=False, fp8_wgrad=False, **OPT)
    if arm in ("hip-fp8sr", "hip-fp8mixsr"):  # stochastically rounded e4m3 activations in the forward
        tr = HipValueTrainer(net, B, lr=lr, device=dev, precision="fp8",
                             fp8_bf16_layers=BF16_LAYERS if arm == "hip-fp8mixsr" else None, **OPT)
        tr.fp8_sr = True
        return tr
    if arm == "hip-fp8mix":  # per-layer precision: BF16_LAYERS in bf16, the rest all-fp8
        return HipValueTrainer(net, B, lr=lr, device=dev, precision="fp8", fp8_bf16_layers=BF16_LAYERS, **OPT)
    return HipValueTrainer(net, B, lr=lr, device=dev, precision="fp8" if arm == "hip-fp8" else "bf16", **OPT)


def heldout_mse(tr, planes, z, B):
    tot, n = 0.0, 0
    for i in range(0, len(planes) - B + 1, B):
        se, _ = tr.evaluate(planes[i:i + B], z[i:i + B])
        tot += float(se)
        n += B
    return tot / max(n, 1)


def grad_cosines(arm_a, arm_b, net, planes, z, B, lr, dev):
    """Per-parameter cosine of one batch's gradients of two trainers at the same weights."""
    ta = make_trainer(arm_a, copy.deepcopy(net), B, lr, dev)
    tb = make_trainer(arm_b, copy.deepcopy(net), B, lr, dev)
    for t in (ta, tb):  # the fp8 trainer calibrates its gradient scales on a first backward
        t.compute_grads(planes[:B], z[:B])
        t.compute_grads(planes[:B], z[:B])
    out = {}
    for name in ta.fp.names:
        a, b = ta.fp.grad_views[name].double().flatten(), tb.fp.grad_views[name].double().flatten()
        out[name] = round(float(torch.nn.functional.cosine_similarity(a, b, dim=0)), 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--positions", type=int, default=65536)
    ap.add_argument("--heldout", type=int, default=8192)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--lr", type=float, default=0.02)
    ap.add_argument("--filters", type=int, default=152)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--arms", default="torch-fp32,hip-bf16,hip-fp8")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--task", default="teacher", choices=["teacher", "material"],
                    help="teacher: a random-init value teacher's outputs; material: tanh of the stone and atari "
                         "balance (data/synthetic.py value_material_pool)")
    ap.add_argument("--init", default="keras", choices=["keras", "he"],
                    help="student init: keras = the reference's uniform(-0.05, 0.05); he = uniform He bounds "
                         "(the reference init shrinks a 12-layer trunk's signal ~30x)")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "momentum", "adam"])
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--decay", type=float, default=0.0, help="Keras lr decay: lr / (1 + decay * step)")
    ap.add_argument("--bf16-layers", default="0,11", help="hip-fp8mix arms: layers kept in bf16")
    ap.add_argument("--seeds", type=int, default=1,
                    help="repeat every arm with this many student inits / batch orders (same data)")
    a = ap.parse_args()
    global BF16_LAYERS
    BF16_LAYERS = tuple(int(x) for x in a.bf16_layers.split(",") if x != "")
    OPT.update(optimizer=a.optimizer, momentum=a.momentum if a.optimizer == "momentum" else 0.0, decay=a.decay)
    dev = torch.device("cuda")
    t0 = time.perf_counter()
    rng = np.random.default_rng(a.seed)
    if a.task == "teacher":
        probe = Preprocess(VALUE_FEATURES).states_to_uint8(random_game_states(2048, rng))
        teacher = value_teacher(49, a.filters, a.layers, device=dev, probe=probe)
        planes, z = value_teacher_pool(a.positions + a.heldout, teacher, seed=a.seed + 1)
        del teacher
    else:
        from alphago_amd.data.synthetic import value_material_pool
        planes, z = value_material_pool(a.positions + a.heldout, seed=a.seed + 1)
    torch.cuda.empty_cache()
    t_data = time.perf_counter() - t0
    print("data: %d positions in %.1f s, target std %.3f" % (len(z), t_data, float(np.std(z))), flush=True)
    P = torch.from_numpy(planes).to(dev)
    Z = torch.from_numpy(z).to(dev)
    Ptr, Ztr = P[:a.positions], Z[:a.positions]
    Pho, Zho = P[a.positions:], Z[a.positions:]
    B = a.batch
    steps = a.positions // B
    res = {"teacher_target_std": round(float(Z.std()), 4), "heldout_var": round(float(Zho.var()), 5)}
    arms = {}
    mid_net = None
    from alphago_amd.models.nets import he_uniform_
    for k in range(a.seeds):
        # the batch order and symmetries of every epoch, shared by all arms of this seed
        g = torch.Generator(device="cpu").manual_seed(a.seed + 7 + 1000 * k)
        orders = [torch.randperm(a.positions, generator=g) for _ in range(a.epochs)]
        syms = [torch.randint(0, 8, (a.positions,), dtype=torch.int32, generator=g) for _ in range(a.epochs)]
        torch.manual_seed(a.seed + 100 + 1000 * k)
        student0 = ValueNet(49, filters_per_layer=a.filters, layers=a.layers)
        if a.init == "he":
            he_uniform_(student0)
        for arm in [x for x in a.arms.split(",") if x]:
            net = copy.deepcopy(student0)
            tr = make_trainer(arm, net, B, a.lr, dev)
            mses, losses = [], []
            t1 = time.perf_counter()
            for e in range(a.epochs):
                ep_loss = 0.0
                order, sym = orders[e].to(dev), syms[e].to(dev)
                for s in range(steps):
                    idx = order[s * B:(s + 1) * B]
                    loss, _ = tr.step(Ptr.index_select(0, idx), Ztr.index_select(0, idx), sym[s * B:(s + 1) * B])
                    ep_loss += float(loss) if s % 16 == 0 else 0.0
                torch.cuda.synchronize()
                losses.append(round(ep_loss / max(1, (steps + 15) // 16) / B, 5))
                mses.append(round(heldout_mse(tr, Pho, Zho, B), 5))
                print("[%s seed %d] epoch %d heldout_mse %.5f train_mse %.5f" % (arm, k, e + 1, mses[-1], losses[-1]),
                      flush=True)
                if arm == "hip-bf16" and e == 0 and k == 0:
                    mid_net = copy.deepcopy(net)
            r = arms.setdefault(arm, {"heldout_mse_seeds": [], "train_mse_seeds": [], "train_s": []})
            r["heldout_mse_seeds"].append(mses)
            r["train_mse_seeds"].append(losses)
            r["train_s"].append(round(time.perf_counter() - t1, 1))
            del tr
            torch.cuda.empty_cache()
    for r in arms.values():
        r["heldout_mse"] = [round(float(np.mean(c)), 5) for c in zip(*r["heldout_mse_seeds"])]
        r["train_mse"] = [round(float(np.mean(c)), 5) for c in zip(*r["train_mse_seeds"])]
        r["heldout_mse_over_var"] = [round(m / float(Zho.var()), 4) for m in r["heldout_mse"]]
    if "torch-fp32" in arms:
        ref = arms["torch-fp32"]["heldout_mse"]
        for arm, r in arms.items():
            r["rel_gap_vs_fp32"] = [round((m - f) / f, 4) for m, f in zip(r["heldout_mse"], ref)]
    res["arms"] = arms
    if mid_net is not None:
        idx = orders[0][:B].to(dev)
        res["grad_cosine_fp8_vs_fp32_after_epoch1"] = grad_cosines("hip-fp8", "torch-fp32", mid_net,
                                                                   Ptr.index_select(0, idx), Ztr.index_select(0, idx),
                                                                   B, a.lr, dev)
        res["grad_cosine_bf16_vs_fp32_after_epoch1"] = grad_cosines("hip-bf16", "torch-fp32", mid_net,
                                                                    Ptr.index_select(0, idx), Ztr.index_select(0, idx),
                                                                    B, a.lr, dev)
    out = {"metric": "value-net held-out MSE on a learnable value task (%dx%d, 49 planes)" % (a.layers, a.filters),
           "task": a.task, "init": a.init, "optimizer": a.optimizer, "decay": a.decay, "seeds": a.seeds,
           "bf16_layers": list(BF16_LAYERS), "positions": a.positions,
           "heldout": a.heldout, "epochs": a.epochs, "batch": B, "lr": a.lr, "data_s": round(t_data, 1),
           "net": "%dx%d" % (a.layers, a.filters), **res}
    print(json.dumps(out), flush=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
