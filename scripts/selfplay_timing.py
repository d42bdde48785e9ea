"""Phase timing of the self-play benchmark loop (benchmarks/selfplay_dp_benchmark.py:
3 moves x 1600 playouts, tree reuse): host phases of BatchedMCTS.search, the
GPU wait, update_with_move, and the leaves evaluated per search round."""
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
    playouts = int(sys.argv[2]) if len(sys.argv) > 2 else 1600
    moves = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda")
    torch.manual_seed(int(os.environ.get("SEED", "0")))  # the benchmark's rank-0 weights
    pol = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=192, layers=12, device=dev)
    val = CNNValue(VALUE_FEATURES, filters_per_layer=152, layers=12, device=dev)
    m = M.BatchedMCTS(pol, val, n_trees=trees, seed=0)
    f = m.forest
    states = [go.GameState() for _ in range(trees)]
    for i, st in enumerate(states):
        st.do_move((3 + i % 13, 3 + (i * 7) % 13))
    m.search(states, 16, 16)
    torch.cuda.synchronize()
    def submit(f, slot, pe, ve):  # BatchedMCTS._submit with its two halves timed
        t = time.perf_counter()
        L = f.n_pending
        s0 = f.leaf_state(0)
        np_ = s0.size * s0.size
        ladder = pe.needs_ladder or (ve is not None and ve.needs_ladder)
        b, a, mm, l = m._enc_buffers(L, np_, slot)
        f.leaf_encode_into(b.data_ptr(), a.data_ptr(), mm.data_ptr(), l.data_ptr() if ladder else 0, b.shape[0],
                           m.threads)
        dt_enc = time.perf_counter() - t
        T["encode"] += dt_enc
        N["encode"] += 1
        if os.environ.get("DUMP_SLOW") and dt_enc > 0.015 and not os.path.exists(os.environ["DUMP_SLOW"]):
            hist = []
            for i in range(L):
                st = f.leaf_state(i)
                hist.append([list(mv) if mv is not None else None for mv in st.history])
            with open(os.environ["DUMP_SLOW"], "w") as fh:
                json.dump({"encode_s": dt_enc, "histories": hist}, fh)
        T["max_leaves"] = max(T["max_leaves"], L)
        t = time.perf_counter()
        lad = l[:L] if ladder else None
        hp = pe.submit_encoded(b[:L], a[:L], mm[:L], lad, slot=slot, to_host=True)
        hv = ve.submit_encoded(b[:L], a[:L], mm[:L], lad, slot=slot, to_host=True) if ve is not None else None
        T["launch"] += time.perf_counter() - t
        return hp, hv
    m._submit = timed("submit", submit)
    m._finish = timed("finish", m._finish)
    pe, ve = m._encoded_engines()
    for eng in {id(pe): pe, id(ve): ve}.values():  # graph captures / bucket creation inside the timed loop
        eng._capture = timed("capture", eng._capture)
        eng._make_bucket = timed("make_bucket", eng._make_bucket)
    out = []
    for k in range(moves):
        T.clear()
        N.clear()
        e0 = m.forest.total_evals
        t = time.perf_counter()
        mv = m.search(states, playouts, 16)
        torch.cuda.synchronize()
        ts = time.perf_counter() - t
        t = time.perf_counter()
        for i, st in enumerate(states):
            if not st.is_end_of_game:
                st.do_move(mv[i])
                m.update_with_move(i, mv[i])
        tu = time.perf_counter() - t
        ev = m.forest.total_evals - e0
        depth = getattr(f, "max_expanded_depth", None)
        out.append({"move": k, "max_depth": depth() if callable(depth) else depth, "search_s": round(ts, 3), "update_s": round(tu, 3), "evals": ev,
                    "leaf_evals_per_s": round(ev / ts), "phases_s": {a: round(b, 3) for a, b in T.items()},
                    "rounds": dict(N)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
