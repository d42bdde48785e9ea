"""Layer-0 (5x5, 48 planes padded to 64) wgrad: padded-channel path vs cin_real=48 path."""
import torch
from alphago_amd import ops
ops.load()
dev = torch.device("cuda")
B, S, F = 1024, 19, 192
M = B * S * S
x0 = ops.padded_empty(B, S, 2, 64, dev); x0[:, 2:21, 2:21, :48].normal_()
dz = ops.padded_empty(B, S, 1, F, dev); dz[:, 1:20, 1:20].normal_()
ns = ops.wgrad_splits(M, 5, 1, 512)
slab = torch.empty(ns, 25, F, 64, device=dev); dbs = torch.zeros(ns, F, device=dev)

def timeit(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3

for rep in range(2):
    t64 = timeit(lambda: ops.conv_wgrad(x0, dz, slab, dbs, 5, S, 2, 1))
    t48 = timeit(lambda: ops.conv_wgrad(x0, dz, slab, dbs, 5, S, 2, 1, cin_real=48))
    print("nsplit %d: padded-64 %.1f us, cin_real-48 %.1f us" % (ns, t64, t48))
