"""Gradient agreement of the fp8 value trainer (fp8 forward, optional fp8 dgrad / wgrad) with the bf16
trainer on the full 12 x 152 value net, B = 256, same weights and batch: per-tensor cosine of the
second backward (the first calibrates the gradient scales).  Prints one JSON line per arm."""
import copy
import json

import torch

from alphago_amd.models.nets import ValueNet
from alphago_amd.train.engine import HipValueTrainer

dev = torch.device("cuda")
torch.manual_seed(0)
B = 256
net = ValueNet(49, filters_per_layer=152, layers=12)
g = torch.Generator().manual_seed(5)
planes = (torch.rand(B, 49, 19, 19, generator=g) < 0.3).to(torch.uint8).to(dev)
z = (torch.randint(0, 2, (B,), generator=g) * 2 - 1).float().to(dev)
t16 = HipValueTrainer(copy.deepcopy(net), B, lr=0.0, device=dev)
for _ in range(2):
    t16.compute_grads(planes, z)
for name, kw in (("fp8_fwd", {"fp8_wgrad": False}), ("fp8_fwd+dgrad", {"fp8_dgrad": True, "fp8_wgrad": False}),
                 ("fp8_fwd+wgrad", {"fp8_wgrad": True}), ("fp8_fwd+dgrad+wgrad", {"fp8_dgrad": True, "fp8_wgrad": True})):
    t8 = HipValueTrainer(copy.deepcopy(net), B, lr=0.0, device=dev, precision="fp8", **kw)
    for _ in range(2):
        t8.compute_grads(planes, z)
    cos = {}
    for n in t8.fp.names:
        a, b = t8.fp.grad_views[n], t16.fp.grad_views[n]
        cos[n] = round(torch.nn.functional.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0).item(), 5)
    trunk = [v for k, v in cos.items() if k[0] in "wb" and k[1:].isdigit()]
    print(json.dumps({"arm": name, "min_trunk_cos": min(trunk), "mean_trunk_cos": round(sum(trunk) / len(trunk), 5),
                      "per_tensor": cos}), flush=True)
