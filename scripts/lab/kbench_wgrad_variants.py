"""3x3 192->192 wgrad at the SL bench batch: production kernel vs kernel-lab variants
(1 = one tap per workgroup, 2 = 256-thread tile, 3 / 4 = LDS ring with 3 / 4 slots), timed
round-robin (the first arm of a process runs at a lower clock), min over rounds."""
import os
import sys
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from alphago_amd import ops  # noqa: E402

ops.load()
lab = ops.lab()
dev = torch.device("cuda")
B, S, F = int(sys.argv[1]) if len(sys.argv) > 1 else 2176, 19, 192
M = B * S * S
x = ops.padded_empty(B, S, 1, F, dev); x[:, 1:20, 1:20].normal_()
dz = ops.padded_empty(B, S, 1, F, dev); dz[:, 1:20, 1:20].normal_()
targets = [int(t) for t in sys.argv[2].split(",")] if len(sys.argv) > 2 else [512]
VARIANTS = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 2, 3, 4]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


arms = {}
for tgt in targets:
    ns = ops.wgrad_splits(M, 9, 1, tgt)
    slab = torch.empty(ns, 9, F, F, device=dev)
    dbs = torch.zeros(ns, F, device=dev)
    for v in VARIANTS:
        fn = (lambda s=slab, d=dbs: ops.conv_wgrad(x, dz, s, d, 3, S, 1, 1)) if v == 0 else \
             (lambda s=slab, d=dbs, v=v: lab.conv_wgrad(x, dz, s, d, 3, S, 1, 1, 0, v))
        arms["t%d v%d (ns %d)" % (tgt, v, ns)] = fn
best = {k: 1e9 for k in arms}
for rnd in range(4):
    for k, fn in arms.items():
        best[k] = min(best[k], timeit(fn))
flop = 2.0 * M * F * F * 9
for k, t in best.items():
    print("%-22s %7.1f us  %6.1f TF/s" % (k, t, flop / t / 1e6), flush=True)
