"""Reinforcement learning of the policy network by self-play
(reference AlphaGo/training/reinforcement_policy_trainer.py).

Each iteration: play ``game_batch_size`` games of the learner against an
opponent drawn uniformly from the pool (on every rank, different seeds), then
one policy-gradient update.  Default loss is REINFORCE as in the paper,
    grad = -1/N * sum_games z_g * sum_t grad log p(a_t | s_t),
with z = +1 for a learner win and -1 for a loss — computed by the fused HIP
head kernel with per-board weights z.  ``--loss reference`` reproduces the
reference's update (one step per game of binary cross-entropy on the softmax
with the learning rate negated for lost games; fused HIP head
kernel or autograd).

Fixes over the reference: per-game learner colour is used for the reward
(Q7), training pairs use the state before the learner's move (Q6), snapshots
are saved every ``save_every`` iterations and added to the opponent pool
(the reference's TODOs at :123,164-175), positional
``initial_weights initial_json`` are honoured.

Fault tolerance (the reference had none): a native checkpoint
(``rl_checkpoint.pt`` in ``--checkpoint-dir``, default ``--model_folder``)
holds the learner's master weights and SGD iteration, the next iteration, the
opponent pool, every rank's RNG states (pool draws / learner colours, both
samplers' move-sampling generators) and the metrics history; ``--resume``
continues bit-identically after a crash (fault hooks ``utils/faults.py`` fire
at iteration granularity), ``--watchdog-timeout`` turns a hang into an exit
for ``torchrun --max-restarts``.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from typing import List, Optional

import numpy as np
import torch

from .. import go
from ..models.policy import CNNPolicy
from ..parallel import dist as agdist
from ..parallel.launch import add_gpus_arg, cli_ranks, exit_status
from ..search.selfplay import BatchedSampler, play_games
from ..utils import faults
from ..utils.metrics import MetricsLogger
from ..utils.watchdog import Watchdog, enable_collective_timeouts
from . import checkpoint as ckpt
from .engine import make_policy_trainer


def rl_update(trainer, records, B: int, device, loss: str = "reinforce", baseline: str = "mean",
              clip_grad_norm: float = 0.0, weight_decay: float = 0.0) -> dict:
    """One policy-gradient step over all learner positions of a batch of games
    (``loss="reference"``: the reference's per-game binary-CE steps instead).

    ``baseline="mean"``: the REINFORCE weight of a position is z - b, with b the mean outcome over all
    learner positions of the iteration (all ranks).  Without it (``"none"``, the paper's form) an iteration
    the learner loses entirely pushes down every move it played and nothing up; at lr 0.01 from a 12 x 192
    SL net that feedback collapsed the policy within one iteration after 34 iterations of gains
    (profiles/r6/README.md).  With the baseline such an iteration does not move the weights.

    ``clip_grad_norm`` > 0: the update's gradient is scaled down to at most this L2 norm, and an update
    with a non-finite gradient is skipped (the weights stay finite).  With the baseline at lr 0.01 the
    gradient norm stayed at 2-6 for 22 iterations, then grew to 65, 373 and 1.6e5 and the weights
    diverged (profiles/r6/README.md).  ``weight_decay``: L2 term wd * w added to the gradient (before the
    clip): the ReLU trunk has no normalisation, and a sharpening policy grows its weights and with them
    the gradient norm (2 -> 100 over 60 iterations at lr 0.003, profiles/r6/README.md)."""
    if loss == "reference":
        return _reference_bce_update(trainer, records, B, device)
    X, T, Z = [], [], []
    for planes, moves, w, c in zip(records.planes, records.moves, records.winners, records.learner_colors):
        if len(moves) == 0:
            continue
        z = 1.0 if w == c else (-1.0 if w == -c else 0.0)
        X.append(planes)
        T.append(moves)
        Z.append(np.full(len(moves), z, np.float32))
    C = trainer.net.trunk.in_planes
    S = trainer.net.board
    if X:
        # device records (play_games on a HIP learner) stay on the device
        X = torch.cat(X) if isinstance(X[0], torch.Tensor) else np.concatenate(X)
        T, Z = np.concatenate(T).astype(np.int32), np.concatenate(Z)
    else:
        X, T, Z = np.zeros((0, C, S, S), np.uint8), np.zeros(0, np.int32), np.zeros(0, np.float32)
    n = len(T)
    n_chunks = int(agdist.all_reduce_max(float((n + B - 1) // B)))
    mean_reward = float(Z.mean()) if n else 0.0
    b = 0.0
    if baseline == "mean":
        tot = torch.tensor([float(Z.sum()) if n else 0.0, float(n)], dtype=torch.float64,
                           device=device if agdist.env().backend == "nccl" else "cpu")
        agdist.all_reduce_sum_(tot)
        b = float(tot[0] / tot[1]) if float(tot[1]) > 0 else 0.0
    elif baseline != "none":
        raise ValueError("baseline must be 'mean' or 'none'")
    scale = float(B) / max(1, n)
    _accumulate_grads(trainer, X, T, (Z - b) * scale, B, device, n_chunks)
    if weight_decay > 0:
        trainer.fp.grad.add_(trainer.fp.flat, alpha=weight_decay)
    gnorm = float(trainer.fp.grad.norm())
    skipped = not math.isfinite(gnorm)
    if skipped:  # every rank sees the same all-reduced gradient, so every rank skips
        trainer.fp.grad.zero_()
    elif clip_grad_norm > 0 and gnorm > clip_grad_norm:
        trainer.fp.grad.mul_(clip_grad_norm / gnorm)
    if not skipped:
        trainer.apply_update()
    return {"positions": n, "mean_reward": mean_reward, "baseline": b, "grad_norm": gnorm, "skipped": skipped}


def _accumulate_grads(trainer, X, T, W, B, device, n_chunks) -> None:
    """trainer.fp.grad <- sum over B-sized chunks of the weighted-loss gradients
    (padding boards carry target -1 and weight 0).  Chunks accumulate locally
    (``compute_grads(reduce=False)``); the sum is all-reduced ONCE."""
    C, S = trainer.net.trunk.in_planes, trainer.net.board
    n_chunks = max(1, n_chunks)
    acc = torch.zeros_like(trainer.fp.grad) if n_chunks > 1 else None
    on_dev = isinstance(X, torch.Tensor)
    for c in range(n_chunks):
        sl = slice(c * B, (c + 1) * B)
        xb, tb, wb = X[sl], T[sl], W[sl]
        pad = B - len(tb)
        if pad:
            if on_dev:
                xb = torch.cat([xb, torch.zeros((pad, C, S, S), dtype=torch.uint8, device=xb.device)])
            else:
                xb = np.concatenate([xb, np.zeros((pad, C, S, S), np.uint8)])
            tb = np.concatenate([tb, np.full(pad, -1, np.int32)])
            wb = np.concatenate([wb, np.zeros(pad, np.float32)])
        xt = xb.to(device) if on_dev else torch.from_numpy(xb).to(device)
        trainer.compute_grads(xt, torch.from_numpy(tb).to(device), None,
                              torch.from_numpy(wb.astype(np.float32)).to(device), reduce=False)
        if acc is not None:
            acc += trainer.fp.grad
    if acc is not None:
        trainer.fp.grad.copy_(acc)
    if agdist.env().distributed:
        agdist.all_reduce_sum_(trainer.fp.grad)


def _reference_bce_update(trainer, records, B, device) -> dict:
    """reinforcement_policy_trainer.py:79-103: for every game, one SGD step of
    model.fit(X, one_hot(y), batch_size=len(X)) with binary cross-entropy on the
    softmax output and the learning rate negated for a lost game.  The sign is
    folded into per-board weights (p -= lr * sign * grad == p -= (sign*lr) * grad)
    and 1/len(game) makes the step the game's mean loss, as Keras' fit does.
    Runs on either backend (fused HIP head with loss_kind=1, or autograd).
    With data parallelism, step k averages game k of every rank."""
    C, S = trainer.net.trunk.in_planes, trainer.net.board
    games = []
    for planes, moves, w, c in zip(records.planes, records.moves, records.winners, records.learner_colors):
        if len(moves):
            games.append((planes, np.asarray(moves, np.int32), 1.0 if w == c else (-1.0 if w == -c else 0.0)))
    n_steps = int(agdist.all_reduce_max(float(len(games))))
    prev = trainer.policy_loss
    trainer.policy_loss = "bce"
    n_pos, rewards = 0, []
    try:
        for k in range(n_steps):
            if k < len(games):
                X, T, z = games[k]
            else:  # this rank has run out of games: contribute a zero gradient
                X, T, z = np.zeros((0, C, S, S), np.uint8), np.zeros(0, np.int32), 0.0
            if isinstance(X, torch.Tensor) and len(T) == 0:
                X = np.zeros((0, C, S, S), np.uint8)
            n = len(T)
            W = np.full(n, z * B / max(1, n), np.float32)
            n_chunks = int(agdist.all_reduce_max(float((n + B - 1) // B)))
            _accumulate_grads(trainer, X, T, W, B, device, n_chunks)
            trainer.apply_update()
            n_pos += n
            if n:
                rewards.append(z)
    finally:
        trainer.policy_loss = prev
    return {"positions": n_pos, "mean_reward": float(np.mean(rewards)) if rewards else 0.0, "steps": n_steps}


def _parser():
    p = argparse.ArgumentParser(description="Perform reinforcement learning to improve given policy network. "
                                            "Second phase of pipeline.")
    p.add_argument("initial_weights", help="Path to file with weights to start from.")
    p.add_argument("initial_json", help="Path to file with initial network params.")
    p.add_argument("--model_folder", default=None, help="where snapshots / the opponent pool are saved")
    p.add_argument("--learning_rate", type=float, default=.03,
                   help="reference default; on a 12x192 teacher-pool SL net with 512-game iterations 0.01 climbs to "
                        "a 74%% win rate against the SL start in 40 iterations while 0.03 degrades it "
                        "(profiles/r6/README.md)")
    p.add_argument("--save_every", type=int, default=500, help="save policy every n mini-batches")
    p.add_argument("--game_batch_size", type=int, default=20, help="games per mini-batch (per rank)")
    p.add_argument("--iterations", type=int, default=20, help="number of mini-batches")
    p.add_argument("--minibatch", type=int, default=256, help="positions per gradient chunk")
    p.add_argument("--temperature", type=float, default=1.0)
    p.add_argument("--max-moves", type=int, default=500)
    p.add_argument("--standard-two-pass", action="store_true",
                   help="end a game after any two consecutive passes (reference rule: only when the "
                        "second pass is black's, go.py:345-348, SURVEY Q9)")
    p.add_argument("--loss", default="reinforce", choices=["reinforce", "reference"])
    p.add_argument("--baseline", default="mean", choices=["mean", "none"],
                   help="reinforce: subtract the iteration's mean outcome from z (none: the paper's plain z)")
    p.add_argument("--clip-grad-norm", type=float, default=0.0,
                   help="reinforce: scale each update's gradient to at most this L2 norm and skip non-finite "
                        "updates (0: off)")
    p.add_argument("--weight-decay", type=float, default=0.0, help="reinforce: L2 weight decay added to the gradient")
    p.add_argument("--eval-every", type=int, default=0,
                   help="every N iterations play --eval-games games against the initial weights (recorded as "
                        "eval_win_rate); the best snapshot is kept as model_folder/best.hdf5 (0: off)")
    p.add_argument("--eval-games", type=int, default=200)
    p.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--metrics", default=None)
    p.add_argument("--verbose", "-v", action="store_true")
    p.add_argument("--checkpoint-dir", default=None,
                   help="where rl_checkpoint.pt is written (default: --model_folder; none: no checkpoints)")
    p.add_argument("--checkpoint-every", type=int, default=1, help="native checkpoint every N iterations")
    p.add_argument("--resume", action="store_true", help="continue from rl_checkpoint.pt if it exists")
    p.add_argument("--watchdog-timeout", type=float, default=0.0,
                   help="exit a rank that makes no progress for this many seconds (0: off)")
    add_gpus_arg(p)
    return p


def run(cmd_line_args: Optional[List[str]] = None) -> dict:
    argv = list(sys.argv[1:] if cmd_line_args is None else cmd_line_args)
    args = _parser().parse_args(argv)
    code = cli_ranks("train-rl", args, argv)
    if code is not None:
        return code
    env = agdist.init_from_env()
    dev = env.device
    rng = np.random.default_rng(args.seed * 7919 + env.rank)
    learner_pol = CNNPolicy.load_model(args.initial_json, device=dev, weights_file=args.initial_weights)
    opp_pol = CNNPolicy.load_model(args.initial_json, device=dev, weights_file=args.initial_weights)
    backend = args.backend
    trainer = make_policy_trainer(learner_pol.model, args.minibatch, args.learning_rate, 0.0, backend=backend,
                                  device=dev)
    learner = BatchedSampler(learner_pol, args.temperature, seed=args.seed * 31 + env.rank)
    opponent = BatchedSampler(opp_pol, args.temperature, seed=args.seed * 37 + env.rank + 1)
    ref_pol = ev_learner = ev_ref = None
    best = {"eval_win_rate": -1.0, "iteration": -1, "path": None}
    if args.eval_every > 0:  # the fixed reference: the initial weights, with evaluation samplers of their own
        ref_pol = CNNPolicy.load_model(args.initial_json, device=dev, weights_file=args.initial_weights)
        ev_learner = BatchedSampler(learner_pol, args.temperature, seed=args.seed * 41 + env.rank + 7)
        ev_ref = BatchedSampler(ref_pol, args.temperature, seed=args.seed * 43 + env.rank + 9)
    pool: List[Optional[str]] = [None]  # None = the initial weights
    folder = args.model_folder
    if folder:
        if env.is_main:
            os.makedirs(folder, exist_ok=True)
        existing = sorted(f for f in os.listdir(folder) if f.startswith("weights.") and f.endswith(".hdf5")) \
            if os.path.isdir(folder) else []
        pool += [os.path.join(folder, f) for f in existing]
        if env.is_main:
            learner_pol.save_model(os.path.join(folder, "model.json"))
    log = MetricsLogger(args.metrics if env.is_main else None)
    history = []
    size = learner_pol.model.board
    ck_dir = args.checkpoint_dir or folder
    ck_path = os.path.join(ck_dir, "rl_checkpoint.pt") if ck_dir else None
    if ck_dir and env.is_main:
        os.makedirs(ck_dir, exist_ok=True)
    start = 0
    state = ckpt.load(ck_path) if (ck_path and args.resume) else None
    if state is not None and "legacy" not in state:
        ckpt.load_trainer_state(trainer, state["trainer"])
        learner_pol.refresh()
        start = int(state["iteration"])
        pool = [None if p == "" else p for p in state["pool"]]
        history = list(state["history"])
        rs = state["rng"][env.rank]
        rng.bit_generator.state = rs["numpy"]
        learner.gen.set_state(rs["learner"])
        opponent.gen.set_state(rs["opponent"])
        if args.verbose and env.is_main:
            print("resumed at iteration %d (pool of %d)" % (start, len(pool)), flush=True)

    def save_checkpoint(next_it):
        mine = {"numpy": rng.bit_generator.state, "learner": learner.gen.get_state(),
                "opponent": opponent.gen.get_state()}
        allr = agdist.all_gather_object(mine) if env.distributed else [mine]
        if env.is_main:
            ckpt.save(ck_path, trainer, iteration=next_it, pool=["" if p is None else p for p in pool],
                      rng=allr, history=history, config=vars(args))

    enable_collective_timeouts()
    wd = Watchdog(ck_dir if args.watchdog_timeout > 0 else None, env.rank, args.watchdog_timeout)
    if args.watchdog_timeout > 0:
        wd.start()
    for it in range(start, args.iterations):
        faults.maybe_inject(it, env.rank)
        t0 = time.perf_counter()
        choice = pool[int(rng.integers(len(pool)))]
        opp_pol.load_weights(choice if choice else args.initial_weights)
        learner_pol.refresh()
        rec = play_games(learner, opponent, args.game_batch_size, size=size, max_moves=args.max_moves, rng=rng,
                         standard_two_pass=args.standard_two_pass)
        info = rl_update(trainer, rec, args.minibatch, dev, args.loss, args.baseline, args.clip_grad_norm,
                         args.weight_decay)
        learner_pol.refresh()
        wins = sum(1 for w, c in zip(rec.winners, rec.learner_colors) if w == c)
        tot = torch.tensor([float(wins), float(len(rec.winners)), float(sum(rec.lengths))], dtype=torch.float64,
                           device=dev if env.backend == "nccl" else "cpu")
        agdist.all_reduce_sum_(tot)
        dt = time.perf_counter() - t0
        row = {"iteration": it, "wins": int(tot[0]), "games": int(tot[1]), "win_rate": float(tot[0] / tot[1]),
               "games_per_s": float(tot[1]) / dt, "moves_per_s": float(tot[2]) / dt, **info}
        if args.eval_every > 0 and (it + 1) % args.eval_every == 0:
            g = args.eval_games
            er = play_games(ev_learner, ev_ref, g, size=size, max_moves=args.max_moves, rng=rng, record=False,
                            learner_colors=[go.BLACK if i % 2 == 0 else go.WHITE for i in range(g)],
                            standard_two_pass=args.standard_two_pass)
            ew = torch.tensor([float(sum(1 for w, c in zip(er.winners, er.learner_colors) if w == c)), float(g)],
                              dtype=torch.float64, device=dev if env.backend == "nccl" else "cpu")
            agdist.all_reduce_sum_(ew)
            row["eval_win_rate"] = float(ew[0] / ew[1])
            if folder and row["eval_win_rate"] > best["eval_win_rate"]:
                best.update(eval_win_rate=row["eval_win_rate"], iteration=it + 1,
                            path=os.path.join(folder, "best.hdf5"))
                if env.is_main:
                    learner_pol.save_weights(best["path"])
                agdist.barrier()
        history.append(row)
        log.log(**row)
        if args.verbose and env.is_main:
            print("Number of wins this batch: {}/{}  ({:.1f} games/s)".format(row["wins"], row["games"],
                                                                             row["games_per_s"]), flush=True)
        if folder and (it + 1) % args.save_every == 0:
            path = os.path.join(folder, "weights.%05d.hdf5" % (it + 1))
            if env.is_main:
                learner_pol.save_weights(path)
            agdist.barrier()
            pool.append(path)
        wd.beat(it)
        if ck_path and ((it + 1) % args.checkpoint_every == 0 or it + 1 == args.iterations):
            save_checkpoint(it + 1)
    wd.stop()
    return {"history": history, "pool": pool, "best": best}


if __name__ == "__main__":
    sys.exit(exit_status(run()))
