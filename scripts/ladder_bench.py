"""GPU vs CPU ladder planes on random 19x19 positions: host encode time with
and without ladder reading, and the device time of ladder_planes."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from alphago_amd import ops  # noqa: E402
from alphago_amd._native import engine  # noqa: E402
from test_gpu_features import random_positions  # noqa: E402

dev = torch.device("cuda:0")
ops.load()
E = engine()
for n in (256, 2048):
    states = random_positions(n, seed=n, max_len=330)
    E.encode_batch(states, True, 16)
    t = time.perf_counter(); b, a, m, lad = E.encode_batch(states, True, 16); t_lad = time.perf_counter() - t
    t = time.perf_counter(); E.encode_batch(states, False, 16); t_nolad = time.perf_counter() - t
    bd, md = torch.from_numpy(b).to(dev), torch.from_numpy(m).to(dev)
    out = torch.empty(bd.shape, dtype=torch.uint8, device=dev)
    for _ in range(3):
        ops.ladder_planes(bd, md, out, 19)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        ops.ladder_planes(bd, md, out, 19)
    torch.cuda.synchronize()
    t_gpu = (time.perf_counter() - t) / 10
    ok = bool(np.array_equal(out.cpu().numpy(), lad))
    print(json.dumps({"boards": n, "host_encode_with_ladders_ms": round(t_lad * 1e3, 2),
                      "host_encode_no_ladders_ms": round(t_nolad * 1e3, 2), "gpu_ladder_ms": round(t_gpu * 1e3, 3),
                      "bit_equal": ok, "ladder_bits": int((lad != 0).sum())}), flush=True)
