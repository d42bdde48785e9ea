"""One production wgrad shape, launched repeatedly for PMC collection (rocprofv3 --pmc):
``w3`` = 192 -> 192 3x3, ``w0`` = layer 0 (5x5, 48 planes padded to 64, cin_real 48).  B = 2176."""
import sys

import torch

from alphago_amd import ops

ops.load()
which = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2176
dev = torch.device("cuda")
S, F = 19, 192
M = B * S * S
dz = ops.padded_empty(B, S, 1, F, dev)
dz[:, 1:20, 1:20].normal_()
if which == "w0":
    K, P, cin, real = 5, 2, 64, 48
else:
    K, P, cin, real = 3, 1, F, 0
x = ops.padded_empty(B, S, P, cin, dev)
x[:, P:P + S, P:P + S, :real or cin].normal_()
ns = ops.wgrad_nsplit(M, F, cin, K, real)
taps = ops.wgrad_plan(F, cin, K, real)[0]
slab = torch.empty(ns, K * K, F, cin, device=dev)
dbs = torch.zeros(ns, F, device=dev)
for _ in range(10):
    ops.conv_wgrad(x, dz, slab, dbs, K, S, P, 1, cin_real=real)
torch.cuda.synchronize()
print(which, "nsplit", ns, "taps", taps)
