"""Policy-head kernel time vs batch: is there a partial second round of workgroups at B=2176?
(8 resident 4-wave workgroups per CU x 256 CUs = 2048 boards in flight.)"""
import json
import torch
from alphago_amd import ops

ops.load()
dev = torch.device("cuda")
S, C = 19, 192
res = {}
for B in (1024, 1536, 2048, 2176, 2304, 3072, 4096):
    y = ops.padded_empty(B, S, 1, C, dev)
    y[:, 1:20, 1:20].normal_()
    w = torch.randn(C, device=dev) * 0.05
    b = torch.zeros(1, device=dev)
    tgt = torch.randint(0, 361, (B,), device=dev, dtype=torch.int32)
    dz = torch.zeros_like(y)
    loss = torch.zeros(B, device=dev)
    corr = torch.zeros(B, device=dev)
    dhead = torch.zeros(B, C + 1, device=dev)
    fn = lambda: ops.policy_head_train(y, w, b, tgt, dz, loss, corr, dhead, S, 1.0)  # noqa: E731
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
    res[B] = round(best, 1)
    print(json.dumps({"B": B, "us": res[B], "ns_per_board": round(best * 1e3 / B, 1)}), flush=True)
