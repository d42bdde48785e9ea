"""value-generate throughput (paper value-data scheme; train/value.py generate_positions): N games of
SL moves, one random move at a uniform ply U <= max_u, RL moves to the end; one recorded position per
game.  Reports positions/s and moves/s for the pipelined native driver (search/lockstep.py) and the
round-3 Python loop.  12 x 192 policy nets, random init (no checkpoints offline), 19 x 19.

Usage: python benchmarks/value_generate_benchmark.py [--games 256] [--drivers native,python]
Prints one JSON line per driver."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alphago_amd.features import DEFAULT_FEATURES  # noqa: E402
from alphago_amd.models.policy import CNNPolicy  # noqa: E402
from alphago_amd.train.value import generate_positions  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--max-u", type=int, default=450)
    ap.add_argument("--max-moves", type=int, default=500)
    ap.add_argument("--filters", type=int, default=192)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--drivers", default="native,python")
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(0)
    sl = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=a.filters, layers=a.layers, device=dev)
    rl = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=a.filters, layers=a.layers, device=dev)
    for driver in a.drivers.split(","):
        nat = driver == "native"
        generate_positions(sl, rl, min(a.games, 64), max_u=a.max_u, max_moves=a.max_moves, seed=1, native=nat)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        planes, z = generate_positions(sl, rl, a.games, max_u=a.max_u, max_moves=a.max_moves, seed=2, native=nat)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"benchmark": "value-generate", "driver": driver, "games": a.games, "positions": len(z),
                          "seconds": round(dt, 3), "positions_per_s": round(len(z) / dt, 1),
                          "games_per_s": round(a.games / dt, 2), "net": "%dx%d" % (a.layers, a.filters)}),
              flush=True)


if __name__ == "__main__":
    main()
