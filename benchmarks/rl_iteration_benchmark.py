"""RL iteration throughput: one iteration = a batch of learner-vs-opponent games played to the end
in lock-step + the REINFORCE update over all learner positions (train/rl.py; reference
reinforcement_policy_trainer.py:16-125).  Reports games/s and learner positions/s per iteration
for host-side records (featurised on the CPU, copied as numpy, re-uploaded per chunk) and device
records (the GPU featurizer's planes of the sampling forward, kept in HBM).

Usage: python benchmarks/rl_iteration_benchmark.py [--games 20,128,512] [--iterations 2]
Prints one JSON line per (games, records) arm."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alphago_amd.features import DEFAULT_FEATURES  # noqa: E402
from alphago_amd.models.policy import CNNPolicy  # noqa: E402
from alphago_amd.search.selfplay import BatchedSampler, play_games  # noqa: E402
from alphago_amd.train.engine import make_policy_trainer  # noqa: E402
from alphago_amd.train.rl import rl_update  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", default="20,128,512")
    ap.add_argument("--iterations", type=int, default=2)
    ap.add_argument("--filters", type=int, default=192)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--minibatch", type=int, default=0,
                    help="REINFORCE chunk (gradients accumulate over chunks, ONE update per iteration, so the "
                         "chunk size does not change the step); 0 = 2048 at >= 128 games/iteration, else 512")
    ap.add_argument("--max-moves", type=int, default=500)
    ap.add_argument("--records", default="host,device")
    ap.add_argument("--drivers", default="native,python",
                    help="native: the pipelined native lock-step driver (search/lockstep.py); python: the round-3 loop")
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(0)
    learner = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=a.filters, layers=a.layers, device=dev)
    opp = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=a.filters, layers=a.layers, device=dev)
    opp.model.load_state_dict(learner.model.state_dict())
    arms = [(d, m) for d in a.drivers.split(",") for m in a.records.split(",")]
    trainers = {}
    for g in [int(x) for x in a.games.split(",")]:
        mb = a.minibatch or (2048 if g >= 128 else 512)
        if mb not in trainers:
            trainers[mb] = make_policy_trainer(learner.model, mb, 0.001, 0.0, device=dev)
        trainer = trainers[mb]
        for driver, mode in arms:
            nat = driver == "native"
            ls = BatchedSampler(learner, 1.0, seed=1)
            os_ = BatchedSampler(opp, 1.0, seed=2)
            rng = np.random.default_rng(3)
            # warm-up iteration (graph captures for the batch sizes, code objects)
            rec = play_games(ls, os_, g, max_moves=a.max_moves, rng=rng, device_records=(mode == "device"),
                             native=nat)
            rl_update(trainer, rec, mb, dev)
            learner.refresh()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t_play = t_upd = 0.0
            games = positions = moves = 0
            for _ in range(a.iterations):
                t0 = time.perf_counter()
                rec = play_games(ls, os_, g, max_moves=a.max_moves, rng=rng, device_records=(mode == "device"),
                                 native=nat)
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                t1 = time.perf_counter()
                info = rl_update(trainer, rec, mb, dev)
                learner.refresh()
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                t2 = time.perf_counter()
                t_play += t1 - t0
                t_upd += t2 - t1
                games += len(rec.winners)
                positions += info["positions"]
                moves += sum(rec.lengths)
            tot = t_play + t_upd
            print(json.dumps({"games_per_iteration": g, "driver": driver, "records": mode, "iterations": a.iterations,
                              "games_per_s": round(games / tot, 2), "learner_positions_per_s": round(positions / tot, 1),
                              "moves_per_s": round(moves / tot, 1), "play_s_per_it": round(t_play / a.iterations, 3),
                              "update_s_per_it": round(t_upd / a.iterations, 3),
                              "positions_per_it": positions // a.iterations, "reinforce_chunk": mb,
                              "net": "%dx%d" % (a.layers, a.filters)}), flush=True)


if __name__ == "__main__":
    main()
