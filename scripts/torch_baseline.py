"""Baseline: the SL policy train step on plain PyTorch-ROCm (MIOpen convs),
to price the hand-written HIP path against.  Not the product path."""
import argparse, json, time
import torch, torch.nn.functional as F
from alphago_amd.models.nets import PolicyNet

ap = argparse.ArgumentParser()
ap.add_argument("--batches", default="128,256,512")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--cl", type=int, default=1)
a = ap.parse_args()
dev = torch.device("cuda")
torch.backends.cudnn.benchmark = True
net = PolicyNet(48, filters_per_layer=192, layers=12).to(dev)
if a.cl:
    net = net.to(memory_format=torch.channels_last)
opt = torch.optim.SGD(net.parameters(), lr=0.003)
for B in [int(b) for b in a.batches.split(",")]:
    x = torch.randint(0, 2, (B, 48, 19, 19), device=dev, dtype=torch.uint8)
    y = torch.randint(0, 361, (B,), device=dev)
    def step():
        xx = x.to(torch.bfloat16)
        if a.cl:
            xx = xx.contiguous(memory_format=torch.channels_last)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = net.logits_torch(xx)
        loss = F.cross_entropy(logits.float(), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    for _ in range(5): step()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(a.steps): step()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / a.steps
    fl = net.flops_per_position() * 3 * B
    print(json.dumps({"B": B, "ms": dt * 1e3, "pos_per_s": B / dt, "TFLOPs": fl / dt / 1e12, "cl": a.cl}), flush=True)
