"""Forward conv time per layer at the SL batch: layer 0 (5x5, 48 planes padded to 64) vs a 3x3 192->192
layer, production tiling.  Sizes the payoff of a 48-channel K loop for layer 0."""
import json
import torch
from alphago_amd import ops

ops.load()
dev = torch.device("cuda")
B, S, F = 2176, 19, 192


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
    return round(best, 1)


x0 = ops.padded_empty(B, S, 2, 64, dev)
x0[:, 2:21, 2:21, :48] = torch.randint(0, 2, (B, 19, 19, 48), device=dev).to(torch.bfloat16)
w0 = torch.randn(F, 48, 5, 5, device=dev) * 0.05
wf0 = ops.packed_weight_like(w0, 64, F)
ops.pack_weights([w0], [wf0])
x1 = ops.padded_empty(B, S, 1, F, dev)
x1[:, 1:20, 1:20].normal_()
w1 = torch.randn(F, F, 3, 3, device=dev) * 0.05
wf1 = ops.packed_weight_like(w1, F, F)
ops.pack_weights([w1], [wf1])
bias = torch.zeros(F, device=dev)
y = ops.padded_empty(B, S, 1, F, dev)
t0 = timeit(lambda: ops.conv_fwd(x0, wf0, bias, y, 5, S, 2, 1))
t1 = timeit(lambda: ops.conv_fwd(x1, wf1, bias, y, 3, S, 1, 1))
M = B * S * S
print(json.dumps({"layer0_5x5_us": t0, "layer0_pf": round(2 * M * F * 25 * 64 / t0 / 1e9, 3),
                  "layer0_pf_useful_48ch": round(2 * M * F * 25 * 48 / t0 / 1e9, 3),
                  "conv3x3_us": t1, "conv3x3_pf": round(2 * M * F * 9 * F / t1 / 1e9, 3)}))
