"""Diagnose HIP-vs-fp32 gradient agreement across small-batch paths (split-K, overlap)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd.models.nets import PolicyNet  # noqa: E402
from alphago_amd.train.engine import HipPolicyTrainer, TorchPolicyTrainer  # noqa: E402

dev = torch.device("cuda")
for B in (8, 16, 32):
    for splitk in ("1", "0"):
        for overlap in (None, False):
            os.environ["ALPHAGO_AMD_SPLITK"] = splitk
            torch.manual_seed(0)
            net = PolicyNet(48, filters_per_layer=192, layers=12)
            ref_net = copy.deepcopy(net)
            g = torch.Generator().manual_seed(5)
            planes = torch.randint(0, 2, (B, 48, 19, 19), dtype=torch.uint8, generator=g).to(dev)
            tgt = torch.randint(0, 361, (B,), dtype=torch.int32, generator=g).to(dev)
            sym = torch.randint(0, 8, (B,), dtype=torch.int32, generator=g).to(dev)
            hip = HipPolicyTrainer(net, B, lr=0.05, device=dev, overlap=overlap)
            ref = TorchPolicyTrainer(ref_net, B, lr=0.05, device=dev)
            hip.compute_grads(planes, tgt, sym)
            ref.compute_grads(planes, tgt, sym)
            torch.cuda.synchronize()
            cos = {}
            for name in hip.fp.names:
                if not name.startswith("w"):
                    continue
                a, b = hip.fp.grad_views[name].double().flatten(), ref.fp.grad_views[name].double().flatten()
                cos[name] = round(torch.nn.functional.cosine_similarity(a, b, dim=0).item(), 5)
            allc = torch.nn.functional.cosine_similarity(hip.fp.grad.double(), ref.fp.grad.double(), dim=0).item()
            print("B=%d splitk=%s overlap=%s(%s) sk_fwd=%s all=%.5f min=%.5f %s" % (
                B, splitk, overlap, hip.overlap, hip.sk_fwd[1], allc, min(cos.values()),
                " ".join("%s:%.4f" % kv for kv in cos.items())), flush=True)
