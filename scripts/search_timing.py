"""Where the batched-MCTS round goes: host phases of BatchedMCTS.search
(gather, encode+submit, wait for the GPU, collect+apply) timed by wrapping the
methods, plus the GPU's own time per evaluation from CUDA events.
Usage: python scripts/search_timing.py [trees] [playouts]"""
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from alphago_amd import go  # noqa: E402
from alphago_amd.features import DEFAULT_FEATURES, VALUE_FEATURES  # noqa: E402
from alphago_amd.models.policy import CNNPolicy, CNNValue  # noqa: E402
from alphago_amd.search import mcts as M  # noqa: E402

T = collections.Counter()
N = collections.Counter()


def timed(name, fn):
    def w(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            T[name] += time.perf_counter() - t
            N[name] += 1
    return w


def main():
    trees = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    playouts = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    dev = torch.device("cuda")
    pol = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=192, layers=12, device=dev)
    val = CNNValue(VALUE_FEATURES, filters_per_layer=152, layers=12, device=dev)
    s = M.BatchedMCTS(pol, val, n_trees=trees, seed=0)
    states = [go.GameState() for _ in range(trees)]
    for i, st in enumerate(states):
        st.do_move((3 + i % 5, 3 + (i // 5) % 5))
    s.search(states, 32, 16)
    torch.cuda.synchronize()
    pe, ve = s._encoded_engines()
    # split _finish into wait (event sync) and the rest
    orig_collect = type(pe).collect

    def collect(self, handle):
        bk, n, ev = handle
        if ev is not None:
            t = time.perf_counter()
            ev.synchronize()
            T["gpu_wait"] += time.perf_counter() - t
            N["gpu_wait"] += 1
        return orig_collect(self, handle)
    type(pe).collect = collect
    if type(ve) is not type(pe):
        type(ve).collect = collect
    s._submit = timed("submit(encode+H2D+launch)", s._submit)
    s._finish = timed("finish(wait+collect+apply)", s._finish)
    # GPU time of one policy+value evaluation of the same size
    f0 = s._forests[0]
    ev0 = s.forest.total_evals
    t0 = time.perf_counter()
    s.search(states, playouts, 16)
    dt = time.perf_counter() - t0
    res = {"trees": trees, "playouts": playouts, "wall_s": round(dt, 3),
           "leaf_evals_per_s": None, "phases_s": {k: round(v, 3) for k, v in T.items()},
           "calls": dict(N)}
    evals = s.forest.total_evals - ev0
    res["leaf_evals_per_s"] = round(evals / dt)
    # pure GPU: replay the evaluation graphs back to back
    L = f0.n_trees * 16
    b, a, m, l = s._enc_buffers(L, 361, 0)
    lad = l[:L] if (pe.needs_ladder or ve.needs_ladder) else None
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        pe.submit_encoded(b[:L], a[:L], m[:L], lad, slot=0)
        ve.submit_encoded(b[:L], a[:L], m[:L], lad, slot=0)
    e0.record()
    for _ in range(10):
        pe.submit_encoded(b[:L], a[:L], m[:L], lad, slot=0)
        ve.submit_encoded(b[:L], a[:L], m[:L], lad, slot=0)
    e1.record()
    torch.cuda.synchronize()
    res["gpu_ms_per_eval_batch"] = round(e0.elapsed_time(e1) / 10, 3)
    res["leaves_per_batch"] = L
    res["gpu_bound_leaf_evals_per_s"] = round(L / (e0.elapsed_time(e1) / 10 / 1e3))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
