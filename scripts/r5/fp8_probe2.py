"""fp8 160-wide forward at B = 1024 (value layer shape): production vs the lab timing probes
(variant 100 + PROBE bits: 1 no MFMA, 2 no pixel loads, 4 no weight staging, 8 no LDS fragment
reads, 16 no epilogue stores; wrong values), round-robin min of 4 rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from alphago_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ops.load()
B = int(os.environ.get("P_B", "1024"))
S, K = 19, 3
C = int(os.environ.get("P_C", "160"))  # 160 (value) or 192 (policy)
x8 = torch.randint(0, 0x38, (B, S + 2, S + 2, C), dtype=torch.uint8, device=dev)
CR = 152 if C == 160 else C
w = torch.randn(CR, CR, K, K, device=dev) * 0.05
w8, ew = ops.pack_weights_fp8(w, C, C)
bias = torch.zeros(C, device=dev)
scales = torch.tensor([127, 127 - ew], dtype=torch.int32, device=dev)
osc = torch.ones(1, device=dev)
amax = ops.fp8_amax_buffer(1, dev)[0]
yb = ops.padded_empty(B, S, 1, C, dev)
y8 = torch.zeros((B, S + 2, S + 2, C), dtype=torch.uint8, device=dev)
# P_OUT: "both" = bf16 + e4m3 outputs; "fp8mb" = the fp8 value-training forward (e4m3 + ReLU' bitmask)
OUT = os.environ.get("P_OUT", "both")
mb = torch.zeros(B * (S + 2) * (S + 2) * ops.mbits_words(C), dtype=torch.int32, device=dev) if OUT == "fp8mb" else None
if OUT in ("fp8mb", "fp8"):  # "fp8": the inference chain's e4m3-only output
    yb = None
variants = [int(v) for v in os.environ.get("P_VARIANTS", "0,101,102,104,108,116,106,114,130,131,117").split(",")]
res = {v: [] for v in variants}


def call(v):
    if v == 0:
        ops.conv_fwd_fp8(x8, w8, bias, scales, osc, K, S, 1, 1, y_bf16=yb, y_fp8=y8, amax=amax, mbits=mb)
    else:
        ops.lab().conv_fwd_fp8(x8, w8, bias, scales, osc, amax, yb, y8, K, S, 1, 1, v, mb)


for v in res:
    for _ in range(10):
        call(v)
torch.cuda.synchronize()
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
print(json.dumps({"B": B, "C": C, "out": OUT, "cw": int(w8.shape[-1]), "us_per_call_min": {v: round(min(t), 1) for v, t in res.items()}}))
