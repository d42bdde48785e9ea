"""conv_wgrad_reduce alone: 12 launches (192 x 192 3x3 slabs, nsplit 9 / 22 / 56) captured in a graph."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
C, T = 192, 9
for ns in (9, 22, 56):
    slabs = [torch.randn(ns, T, C, C, device=dev) for _ in range(2)]
    dbs = [torch.randn(ns, C, device=dev) for _ in range(2)]
    gw = [torch.zeros(C, C, 3, 3, device=dev) for _ in range(12)]
    gb = [torch.zeros(C, device=dev) for _ in range(12)]

    def chain():
        for l in range(12):
            ops.conv_wgrad_reduce(slabs[l % 2], dbs[l % 2], gw[l], gb[l], 1.0, 0.0)
    chain()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        chain()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    e1.synchronize()
    print(json.dumps({"nsplit": ns, "us_per_reduce": round(e0.elapsed_time(e1) / 20 / 12 * 1e3, 2),
                      "slab_mb": round(ns * T * C * C * 4 / 1e6, 1)}), flush=True)
