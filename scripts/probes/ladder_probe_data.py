"""Write boards + meta + CPU ladder bits for scripts/probes/ladder_probe.hip:
python scripts/probes/ladder_probe_data.py scripts/probes/data"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from alphago_amd._native import engine  # noqa: E402
from test_gpu_features import eye_chain_positions, random_positions  # noqa: E402

os.makedirs(sys.argv[1], exist_ok=True)
sets = {"eye": eye_chain_positions()[-2:], "rand48": random_positions(48, seed=11),
        "rand2048": random_positions(2048, seed=2048, max_len=330)}
for name, states in sets.items():
    b, _, m, lad = engine().encode_batch(states, True, 8)
    with open(os.path.join(sys.argv[1], name + ".bin"), "wb") as f:
        f.write(np.array([b.shape[0], 19], np.int32).tobytes())
        f.write(b.astype(np.int8).tobytes())
        f.write(m.astype(np.int32).tobytes())
        f.write(lad.astype(np.uint8).tobytes())
