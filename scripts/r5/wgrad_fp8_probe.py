"""fp8 wgrad of the 160-wide value layer at B = 1024: production vs lab timing probes (PROBE bits:
1 no MFMA, 2 no staging loads, 4 no LDS fragment reads, 8 no partial-tile stores; wrong values),
round-robin min of 4 rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from alphago_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ops.load()
B = int(os.environ.get("P_B", "1024"))
S, K, C = 19, 3, 160
M = B * S * S
x8 = torch.randint(0, 0x38, (B, S + 2, S + 2, C), dtype=torch.uint8, device=dev)
dz8 = torch.randint(0, 0x38, (B, S + 2, S + 2, C), dtype=torch.uint8, device=dev)
ns = ops.wgrad_fp8_nsplit(M, 3)
slab = torch.zeros(ns, 9, C, C, device=dev)
dbs = torch.zeros(ns, C, device=dev)
xs = torch.tensor([127], dtype=torch.int32, device=dev)
gs = torch.tensor([127], dtype=torch.int32, device=dev)
gm = torch.ones(1, device=dev)
amax = ops.fp8_amax_buffer(1, dev)[0]
probes = [int(v) for v in os.environ.get("P_PROBES", "0,1,2,4,8,3,5,6,7,14,15").split(",")]
res = {p: [] for p in probes}


def call(p):
    ops.lab().conv_wgrad_fp8(x8, dz8, slab, dbs, xs, gs, gm, K, S, 1, 1, amax, p)


for p in res:
    for _ in range(5):
        call(p)
torch.cuda.synchronize()
for _ in range(4):
    for p in res:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(30):
            call(p)
        e1.record()
        torch.cuda.synchronize()
        res[p].append(e0.elapsed_time(e1) / 30 * 1e3)
print(json.dumps({"B": B, "nsplit": ns, "us_per_call_min": {p: round(min(t), 1) for p, t in res.items()}}))
