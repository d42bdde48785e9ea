"""Eager vs HIP-graph-captured SL training steps across minibatch sizes.

The reference trains with minibatch 16 (supervised_policy_trainer.py:93) and
RL fits one game at a time (reinforcement_policy_trainer.py:102): at such sizes
the ~60 kernel launches of a step, not the GPU, set the pace.  Prints one JSON
line per (batch, mode): positions/s, ms/step and host enqueue ms/step.

    python benchmarks/graph_step_benchmark.py --batches 16,64,256,2176
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from alphago_amd.models.nets import PolicyNet  # noqa: E402
from alphago_amd.train.engine import HipPolicyTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="16,64,256,2176")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for B in [int(x) for x in a.batches.split(",")]:
        steps = max(10, a.steps if B <= 256 else a.steps // 5)
        for graph in (False, True):
            torch.manual_seed(0)
            tr = HipPolicyTrainer(PolicyNet(48, filters_per_layer=192, layers=12), B, lr=0.003, device=dev)
            if graph:
                tr.enable_graphs()
            g = torch.Generator(device=dev)
            g.manual_seed(1)
            pool = torch.randint(0, 2, (max(B, 256) * 4, 48, 19, 19), dtype=torch.uint8, device=dev, generator=g)
            tg = torch.randint(0, 361, (pool.shape[0],), dtype=torch.int32, device=dev, generator=g)
            syms = torch.randint(0, 8, (4, B), dtype=torch.int32, device=dev, generator=g)
            idxs = [torch.arange(k * B, (k + 1) * B, device=dev) % pool.shape[0] for k in range(4)]
            # every step gathers its batch from the device pool (the same data movement in both
            # modes); graph mode gathers straight into the captured step's input buffers
            static = tr.static_inputs(pool[:B], tg[:B], syms[0]) if graph else None

            def step(k):
                idx = idxs[k % 4]
                if static is None:
                    tr.step(pool.index_select(0, idx), tg.index_select(0, idx), syms[k % 4].clone())
                else:
                    torch.index_select(pool, 0, idx, out=static[0])
                    torch.index_select(tg, 0, idx, out=static[1])
                    static[2].copy_(syms[k % 4])
                    tr.step(*static)

            for k in range(a.warmup):
                step(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                step(k)
            th = time.perf_counter() - t0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"batch": B, "graph": graph, "positions_per_s": round(steps * B / dt, 1),
                              "ms_per_step": round(dt / steps * 1e3, 3),
                              "host_ms_per_step": round(th / steps * 1e3, 3)}), flush=True)
            del tr, pool


if __name__ == "__main__":
    main()
