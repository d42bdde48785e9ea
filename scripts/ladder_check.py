"""GPU ladder_planes vs the CPU ladder reader on the GPU feature tests'
positions: mismatch report (bit 2 = search budget exhausted on the device)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from alphago_amd import ops  # noqa: E402
from alphago_amd._native import engine  # noqa: E402
from test_gpu_features import eye_chain_positions, random_positions  # noqa: E402

dev = torch.device("cuda:0")
ops.load()
for name, states in (("eye", eye_chain_positions()[-2:]), ("rand48", random_positions(48, seed=11)),
                     ("rand2048", random_positions(2048, seed=2048, max_len=330))):
    b, _, m, lad = engine().encode_batch(states, True, 8)
    bd, md = torch.from_numpy(b).to(dev), torch.from_numpy(m).to(dev)
    out = torch.empty(bd.shape, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    ops.ladder_planes(bd, md, out, 19)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    got = out.cpu().numpy()
    bad = np.argwhere(got != lad)
    print(name, "boards", len(states), "ms %.2f" % (dt * 1e3), "mismatches", len(bad), "budget", int(((got & 4) != 0).sum()),
          [(int(i), int(p), int(got[i, p]), int(lad[i, p])) for i, p in bad[:8]], flush=True)
