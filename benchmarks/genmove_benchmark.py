"""Single-tree genmove latency through the GTP engine (reference: batch-1 policy calls in the serial
search, AlphaGo/mcts.py:107-118; GTP front-end interface/gtp_wrapper.py): an MCTS player (one tree,
1600 playouts, leaf batches of --leaves) on the 12 x 192 policy and 12 x 152 value nets (random init,
no checkpoints offline), answering GTP ``genmove`` on an empty 19 x 19 board and after a few moves.
Reports milliseconds per genmove and leaf evaluations per second.

--positions benchmarks/data/lee_sedol_positions.json: one genmove on each position of the reference's
Lee Sedol game records (every 20th move, scripts/make_genmove_positions.py) instead, with the mean,
median, p95 and max; --ladder-cache 0 turns the search's ladder cache off (A/B).

Usage: python benchmarks/genmove_benchmark.py [--playouts 1600] [--leaves 16,32] [--moves 4]
       [--positions FILE [--max-positions N]] [--ladder-cache 0|1]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alphago_amd.features import DEFAULT_FEATURES, VALUE_FEATURES  # noqa: E402
from alphago_amd.gtp.engine import GTPEngine  # noqa: E402
from alphago_amd.models.policy import CNNPolicy, CNNValue  # noqa: E402
from alphago_amd.search.players import MCTSPlayer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--playouts", type=int, default=1600)
    ap.add_argument("--leaves", default="16,32")
    ap.add_argument("--moves", type=int, default=4, help="genmoves timed per configuration")
    ap.add_argument("--positions", default="", help="JSON of game positions (one genmove each)")
    ap.add_argument("--max-positions", type=int, default=0)
    ap.add_argument("--ladder-cache", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(0)
    pol = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=192, layers=12, device=dev)
    val = CNNValue(VALUE_FEATURES, filters_per_layer=152, layers=12, device=dev)
    if a.positions:
        return positions_mode(a, pol, val, dev)
    for leaves in [int(x) for x in a.leaves.split(",")]:
        player = MCTSPlayer(pol, val, n_playout=a.playouts, leaves_per_batch=leaves)
        player.search.forest.ladder_cache = bool(a.ladder_cache)
        eng = GTPEngine(player)
        eng.send("boardsize 19")
        eng.send("clear_board")
        eng.send("genmove b")  # warm-up: graph captures for the leaf-batch buckets
        eng.send("clear_board")
        times = []
        color = "b"
        for _ in range(a.moves):
            t0 = time.perf_counter()
            reply = eng.send("genmove " + color)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            assert reply.startswith("="), reply
            color = "w" if color == "b" else "b"
        ms = 1000.0 * sum(times) / len(times)
        print(json.dumps({"benchmark": "gtp genmove (single tree)", "playouts": a.playouts, "leaves_per_batch": leaves,
                          "ms_per_genmove": round(ms, 1), "ms_each": [round(1000 * t, 1) for t in times],
                          "leaf_evals_per_s": round(a.playouts / (ms / 1000.0), 1), "ladder_cache": bool(a.ladder_cache),
                          "nets": "policy 12x192 + value 12x152"}), flush=True)


def positions_mode(a, pol, val, dev):
    from alphago_amd import go

    data = json.load(open(a.positions))
    pos = data["positions"][: a.max_positions or None]
    states = []
    for p in pos:
        gs = go.GameState(data["size"])
        for x, y, c in p["moves"]:
            gs.do_move(go.PASS_MOVE if x < 0 else (x, y), c)
        states.append(gs)
    for leaves in [int(x) for x in a.leaves.split(",")]:
        player = MCTSPlayer(pol, val, n_playout=a.playouts, leaves_per_batch=leaves)
        player.search.forest.ladder_cache = bool(a.ladder_cache)
        player.get_move(go.GameState(data["size"]))  # warm-up: graph captures for the leaf-batch buckets
        player.get_move(states[0])
        times = []
        for gs in states:
            t0 = time.perf_counter()
            player.get_move(gs)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            times.append(1000.0 * (time.perf_counter() - t0))
        t = np.array(times)
        print(json.dumps({"benchmark": "genmove on game positions (single tree)", "positions": a.positions,
                          "n_positions": len(t), "playouts": a.playouts, "leaves_per_batch": leaves,
                          "ladder_cache": bool(a.ladder_cache),
                          "ms_mean": round(float(t.mean()), 1), "ms_median": round(float(np.median(t)), 1),
                          "ms_p95": round(float(np.percentile(t, 95)), 1), "ms_max": round(float(t.max()), 1),
                          "p95_over_median": round(float(np.percentile(t, 95) / np.median(t)), 3),
                          "ms_each": [round(v, 1) for v in times],
                          "where": [p["game"] + ":" + str(p["move_number"]) for p in pos],
                          "nets": "policy 12x192 + value 12x152"}), flush=True)


if __name__ == "__main__":
    main()
