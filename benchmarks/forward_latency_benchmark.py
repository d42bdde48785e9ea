"""GPU time of one policy / value forward at small batches (the search's leaf batches, the reference's
batch-1 policy calls in mcts.py:107-118): the HIP-graph evaluate of the inference engines, bf16 and fp8,
timed with device events around each call (median of N calls; planes already on the device, so the
time is the graph's: input pack, 12 convs, head).  Prints one JSON line per (net, precision, batch)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alphago_amd.models.inference import HipTrunkInference, HipValueInference  # noqa: E402
from alphago_amd.models.nets import PolicyNet, ValueNet  # noqa: E402


def gpu_ms(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,4,8,16,32")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    nets = {"policy": (PolicyNet(48, filters_per_layer=192, layers=12).to(dev), HipTrunkInference, 48),
            "value": (ValueNet(49, filters_per_layer=152, layers=12).to(dev), HipValueInference, 49)}
    g = torch.Generator(device=dev).manual_seed(1)
    for name, (net, cls, C) in nets.items():
        for prec in ("bf16", "fp8"):
            eng = cls(net, dev, precision=prec)
            for B in [int(b) for b in a.batches.split(",")]:
                planes = torch.randint(0, 2, (B, C, 19, 19), dtype=torch.uint8, device=dev, generator=g)
                ms = gpu_ms(lambda: eng.evaluate(planes), a.iters)
                print(json.dumps({"net": name, "precision": prec, "batch": B, "gpu_us_per_forward": round(ms * 1e3, 1),
                                  "evals_per_s": round(B / ms * 1e3)}), flush=True)


if __name__ == "__main__":
    main()
