"""Featurisation throughput (reference benchmarks/preprocessing_benchmark.py ran
cProfile over one game; reference code measured 265 positions/s for 46 planes,
BASELINE.md (B)).  Replays the fixture SGFs and featurises every position with the
native featurizer, single-threaded and batched-multithreaded.  Prints JSON."""
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from alphago_amd import go  # noqa: E402
from alphago_amd.features import ALL_NO_LADDER_FEATURES, DEFAULT_FEATURES, Preprocess  # noqa: E402
from alphago_amd.utils.gorecords import sgf_iter_states  # noqa: E402


def positions(sgf_dir):
    out = []
    for f in sorted(glob.glob(os.path.join(sgf_dir, "*.sgf"))):
        try:
            for st, mv, _ in sgf_iter_states(open(f).read()):
                if mv is not None:
                    out.append(st.copy())
        except go.IllegalMove:
            pass
    return out


def gpu_featurizer(states, B=1024, iters=50):
    """Device featurizer: host encode (C++) + H2D + kernel, and the kernel alone."""
    import torch

    from alphago_amd import ops
    from alphago_amd.ops.gpu_features import GpuFeaturizer

    batch = (states * (B // max(1, len(states)) + 1))[:B]
    out = {}
    for name, feats in (("46_planes", ALL_NO_LADDER_FEATURES), ("48_planes_with_ladders", DEFAULT_FEATURES)):
        fz = GpuFeaturizer(feats)
        dev = fz.device
        enc = fz.to_device(fz.encode(batch))
        x = ops.padded_empty(B, 19, 2, 64, dev)
        sens = torch.empty((B, 361), dtype=torch.uint8, device=dev)
        for _ in range(3):
            fz.run(*enc, nhwc=x, P=2, sensible=sens)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            fz.run(*enc, nhwc=x, P=2, sensible=sens)
        torch.cuda.synchronize()
        kern = (time.perf_counter() - t) / iters
        t = time.perf_counter()
        for _ in range(5):
            e = fz.to_device(fz.encode(batch))
            fz.run(*e, nhwc=x, P=2, sensible=sens)
        torch.cuda.synchronize()
        full = (time.perf_counter() - t) / 5
        out[name] = {"batch": B, "kernel_us": round(kern * 1e6, 1), "kernel_pos_per_s": round(B / kern),
                     "encode_h2d_kernel_pos_per_s": round(B / full)}
    return out


def main():
    sgf_dir = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tests/test_data/sgf"
    if not os.path.isdir(sgf_dir):  # synthetic fallback: random games
        import random
        states, gs, rnd = [], go.GameState(), random.Random(0)
        for _ in range(1000):
            moves = gs.get_legal_moves()
            if not moves or gs.is_end_of_game:
                gs = go.GameState()
                continue
            gs.do_move(rnd.choice(moves))
            states.append(gs.copy())
    else:
        states = positions(sgf_dir)
    res = {"positions": len(states)}
    for name, feats in (("46_planes", ALL_NO_LADDER_FEATURES), ("48_planes_with_ladders", DEFAULT_FEATURES)):
        pp = Preprocess(feats)
        t = time.perf_counter()
        for s in states:
            pp.state_to_uint8(s)
        single = len(states) / (time.perf_counter() - t)
        t = time.perf_counter()
        pp.states_to_uint8(states, threads=8)
        batched = len(states) / (time.perf_counter() - t)
        res[name] = {"single_thread_pos_per_s": round(single), "batched_8_threads_pos_per_s": round(batched),
                     "vs_reference_265_pos_per_s": round(single / 265.0, 1)}
    import torch
    if torch.cuda.is_available():
        res["gpu"] = gpu_featurizer(states)
    t = time.perf_counter()
    n = 0
    for s in states[:200]:
        s.copy().get_legal_moves()
        n += 1
    res["get_legal_moves_us"] = round((time.perf_counter() - t) / max(1, n) * 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
