"""Batched MCTS and self-play throughput on the GPU (policy 12x192, 48 planes;
value 12x152 49 planes; random-init weights).  The reference MCTS made one
batch-1 network call per tree level and ran 10^4 serial simulations per move
(mcts.py:142-161).  Prints JSON: leaf evaluations/s, simulations/s, and
self-play games/s + moves/s for lock-step batched games."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alphago_amd import go  # noqa: E402
from alphago_amd.features import DEFAULT_FEATURES, VALUE_FEATURES  # noqa: E402
from alphago_amd.models.policy import CNNPolicy, CNNValue  # noqa: E402
from alphago_amd.search.mcts import BatchedMCTS  # noqa: E402
from alphago_amd.search.selfplay import BatchedSampler, play_games  # noqa: E402


def main():
    # ALPHAGO_AMD_PRECISION=fp8 runs the policy/value engines on the e4m3 MFMA path
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    small = dev.type == "cpu"
    F, L = (16, 2) if small else (192, 12)
    pol = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=F, layers=L, device=dev)
    val = CNNValue(VALUE_FEATURES, filters_per_layer=152 if not small else F, layers=L, device=dev)  # reference K=152
    trees = int(sys.argv[1]) if len(sys.argv) > 1 else (4 if small else 256)  # 256 trees x 16 leaves saturate the GPU better than 64 (150k vs 49k evals/s bf16)
    playouts = int(sys.argv[2]) if len(sys.argv) > 2 else (32 if small else 800)
    lpt = 16
    s = BatchedMCTS(pol, val, n_trees=trees, seed=0)
    states = [go.GameState() for _ in range(trees)]
    for i, st in enumerate(states):  # a few opening moves so trees differ
        st.do_move((3 + i % 5, 3 + (i // 5) % 5))
    s.search(states, 32, lpt)  # warm-up: HIP graphs per bucket
    if dev.type == "cuda":
        torch.cuda.synchronize()
    e0 = s.forest.total_evals
    t = time.perf_counter()
    s.search(states, playouts, lpt)
    dt = time.perf_counter() - t
    evals = s.forest.total_evals - e0
    if dev.type == "cuda":  # the same search without the two-forest pipeline
        s1 = BatchedMCTS(pol, val, n_trees=trees, seed=0, pipeline=False)
        s1.search(states, 32, lpt)
        torch.cuda.synchronize()
        e1 = s1.forest.total_evals
        t1 = time.perf_counter()
        s1.search(states, playouts, lpt)
        np_evals = (s1.forest.total_evals - e1) / (time.perf_counter() - t1)
    else:
        np_evals = None
    res = {"device": str(dev), "precision": os.environ.get("ALPHAGO_AMD_PRECISION", "bf16"), "trees": trees,
           "leaf_evals_per_s_no_pipeline": round(np_evals) if np_evals else None, "playouts_per_tree": playouts, "leaves_per_tree_per_round": lpt,
           "leaf_evals_per_s": round(evals / dt), "simulations_per_s": round(trees * playouts / dt),
           "seconds_per_move_all_trees": round(dt, 3)}
    games = int(sys.argv[3]) if len(sys.argv) > 3 else (8 if small else 256)
    a, b = BatchedSampler(pol, seed=1), BatchedSampler(pol, seed=2)
    play_games(a, b, min(games, 8), max_moves=20, record=False)  # warm-up
    for record in (False, True):  # record=True also featurises the learner's planes on the host
        t = time.perf_counter()
        rec = play_games(a, b, games, max_moves=722, record=record, rng=np.random.default_rng(0))
        dt = time.perf_counter() - t
        key = "selfplay_recorded" if record else "selfplay"
        res[key] = {"games": games, "games_per_s": round(games / dt, 2), "moves_per_s": round(sum(rec.lengths) / dt),
                    "mean_game_length": float(np.mean(rec.lengths))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
