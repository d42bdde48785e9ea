"""Batched network evaluation throughput (policy 12x192 / 48 planes, value
12x152 / 49 planes) on the HIP engines: bf16 vs fp8 (e4m3 block-scaled MFMA),
uint8-plane input vs the encoded-board input with the GPU featurizer in the
graph.  Replaces the reference's batch-1 Theano forward per state
(policy.py:26-42).  Prints JSON: evaluations/s per configuration."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alphago_amd import go  # noqa: E402
from alphago_amd._native import engine  # noqa: E402
from alphago_amd.features import DEFAULT_FEATURES, VALUE_FEATURES  # noqa: E402
from alphago_amd.models.inference import HipTrunkInference, HipValueInference  # noqa: E402
from alphago_amd.models.nets import PolicyNet, ValueNet  # noqa: E402


def states(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        gs = go.GameState()
        for _ in range(int(rng.integers(10, 200))):
            mv = gs.get_legal_moves(include_eyes=False)
            if not mv:
                break
            gs.do_move(mv[int(rng.integers(len(mv)))])
        out.append(gs)
    return out


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    pnet = PolicyNet(48, filters_per_layer=192, layers=12).to(dev)
    vnet = ValueNet(49, filters_per_layer=152, layers=12).to(dev)
    base = states(256)
    res = {}
    for B in (256, 1024):
        st = (base * (B // len(base) + 1))[:B]
        enc = engine().encode_batch(st, True, 8)
        planes = torch.from_numpy(engine().featurize_batch(st, DEFAULT_FEATURES, 8)).to(dev)
        vplanes = torch.from_numpy(engine().featurize_batch(st, VALUE_FEATURES, 8)).to(dev)
        for prec in ("bf16", "fp8"):
            pe = HipTrunkInference(pnet, dev, feature_list=DEFAULT_FEATURES, precision=prec)
            ve = HipValueInference(vnet, dev, feature_list=VALUE_FEATURES, precision=prec)
            dt = timeit(lambda: pe.evaluate(planes))
            res["policy_%s_B%d_planes" % (prec, B)] = round(B / dt)
            dt = timeit(lambda: pe.evaluate_encoded(*enc))
            res["policy_%s_B%d_encoded" % (prec, B)] = round(B / dt)
            dt = timeit(lambda: ve.evaluate(vplanes))
            res["value_%s_B%d_planes" % (prec, B)] = round(B / dt)
    print(json.dumps({"evals_per_s": res, "note": "encoded = GPU featurizer inside the HIP graph (incl. H2D of the "
                      "2-byte/point encoding; host ladder reading excluded)"}))


if __name__ == "__main__":
    main()
