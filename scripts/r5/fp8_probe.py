"""fp8 160-wide forward at B = 1024 (value layer shape): production vs the coalesced-operand probe
(lab variant 7, wrong values), both chunk widths, round-robin min of 4 rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from alphago_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ops.load()
B, S, K, C = 1024, 19, 3, 160
x8 = torch.randint(0, 0x38, (B, S + 2, S + 2, C), dtype=torch.uint8, device=dev)
w = torch.randn(152, 152, K, K, device=dev) * 0.05
w8, ew = ops.pack_weights_fp8(w, C, C)
bias = torch.zeros(C, device=dev)
scales = torch.tensor([127, 127 - ew], dtype=torch.int32, device=dev)
osc = torch.ones(1, device=dev)
amax = ops.fp8_amax_buffer(1, dev)[0]
yb = ops.padded_empty(B, S, 1, C, dev)
y8 = torch.zeros((B, S + 2, S + 2, C), dtype=torch.uint8, device=dev)
res = {v: [] for v in (0, 7)}


def call(v):
    if v == 0:
        ops.conv_fwd_fp8(x8, w8, bias, scales, osc, K, S, 1, 1, y_bf16=yb, y_fp8=y8, amax=amax)
    else:
        ops.lab().conv_fwd_fp8(x8, w8, bias, scales, osc, amax, yb, y8, K, S, 1, 1, v)


for v in res:
    for _ in range(20):
        call(v)
for _ in range(4):
    for v in res:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(50):
            call(v)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 50 * 1e3)
print(json.dumps({"cw": int(w8.shape[-1]) if w8.dim() else None, "us_per_call_min": {v: round(min(t), 1) for v, t in res.items()}}))
