"""SL fp8-forward trainer diagnosis: per-step loss / accuracy / weight norm at B = 256, lr 0.05,
random-init 12 x 192 policy on a teacher-labelled pool (as scripts/sl_teacher_accuracy.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd.models.nets import PolicyNet  # noqa: E402
from alphago_amd.train.engine import HipPolicyTrainer  # noqa: E402
from alphago_amd.data.synthetic import teacher_pool  # noqa: E402
from alphago_amd.features import DEFAULT_FEATURES  # noqa: E402
from alphago_amd.models.policy import CNNPolicy  # noqa: E402

dev = torch.device("cuda")
prec = sys.argv[1] if len(sys.argv) > 1 else "fp8"
torch.manual_seed(0)
teacher = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=192, layers=12, device=dev)
planes, tgt = teacher_pool(8192, teacher, seed=1)
planes, tgt = torch.from_numpy(planes).to(dev), torch.from_numpy(tgt).to(dev)
net = PolicyNet(48, filters_per_layer=192, layers=12)
tr = HipPolicyTrainer(net, 256, lr=0.05, device=dev, precision=prec)
g = torch.Generator(device=dev).manual_seed(2)
for step in range(60):
    idx = torch.randint(0, planes.shape[0], (256,), device=dev, generator=g)
    loss, corr = tr.step(planes[idx], tgt[idx])
    if step % 5 == 0 or step < 5:
        torch.cuda.synchronize()
        rec = {"step": step, "loss": float(loss) / 256, "acc": float(corr) / 256,
               "wnorm": float(tr.fp.flat.norm()), "gnorm": float(tr.fp.grad.norm())}
        if prec == "fp8":
            rec["scales"] = tr.scales8[:, 0].tolist()
            rec["osc"] = [round(v, 4) for v in tr.osc8.tolist()]
        print(json.dumps(rec), flush=True)
