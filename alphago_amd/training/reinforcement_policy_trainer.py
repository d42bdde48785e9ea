"""Reference module path ``AlphaGo.training.reinforcement_policy_trainer`` (:16-176).

* ``make_training_pairs(player, opp, features, mini_batch_size)`` -- plays
  ``mini_batch_size`` games in lock-step (batched HIP inference) and returns the
  learner's (state planes, one-hot move) pairs per game and the winners, with
  the learner's colour drawn per game (Q7) and its planes taken before its own
  move (Q6).  ``player`` / ``opp`` are policy players (``.policy`` = CNNPolicy)
  or CNNPolicy objects.
* ``train_batch(player, X_list, y_list, winners, lr)`` -- the reference's
  per-game binary-CE update with the learning rate signed by the outcome
  (loss ``reference``); ``alphago_amd.train.rl`` also offers REINFORCE.
* ``run`` -- the CLI (``alphago_amd.train.rl.run``)."""
import numpy as np

from ..search.selfplay import BatchedSampler, play_games
from ..train.rl import run


def _policy(p):
    return getattr(p, "policy", p)


def make_training_pairs(player, opp, features, mini_batch_size, board_size=19, max_moves=500, seed=None):
    pol = _policy(player)
    learner = BatchedSampler(pol, seed=seed or 0)
    opponent = BatchedSampler(_policy(opp), seed=(seed or 0) + 1)
    rec = play_games(learner, opponent, mini_batch_size, size=board_size, max_moves=max_moves,
                     rng=np.random.default_rng(seed))
    X_list, y_list = [], []
    n2 = board_size * board_size
    for planes, moves in zip(rec.planes, rec.moves):
        X_list.append(planes.astype(np.float32))
        y = np.zeros((len(moves), n2), np.float32)
        y[np.arange(len(moves)), moves] = 1.0
        y_list.append(y)
    # winners from each learner's point of view: +1 win, -1 loss, 0 tie
    winners = [int(np.sign(w * c)) for w, c in zip(rec.winners, rec.learner_colors)]
    return X_list, y_list, winners


def train_batch(player, X_list, y_list, winners, lr, trainer=None):
    """One reference-style RL update per game: binary CE on the softmax,
    learning rate +lr for a won game and -lr for a lost one."""
    from ..train.engine import make_policy_trainer
    import torch

    pol = _policy(player)
    if trainer is None:
        n = max(1, max(len(x) for x in X_list) if X_list else 1)
        trainer = make_policy_trainer(pol.model, n, lr, 0.0, device=pol.device)
        trainer.policy_loss = "bce"
    for X, y, w in zip(X_list, y_list, winners):
        if len(X) == 0 or w == 0:
            continue
        planes = torch.as_tensor(np.asarray(X), dtype=torch.uint8, device=pol.device)
        tgt = torch.as_tensor(np.argmax(y, axis=1), dtype=torch.int32, device=pol.device)
        B = trainer.batch
        weight = torch.full((B,), float(w), device=pol.device)
        for i in range(0, len(planes), B):
            p, t = planes[i:i + B], tgt[i:i + B]
            if len(p) < B:  # pad to the engine's fixed batch with zero-weight boards
                pad = B - len(p)
                p = torch.cat([p, p[:1].expand(pad, *p.shape[1:])])
                t = torch.cat([t, t[:1].expand(pad)])
                wt = weight.clone()
                wt[B - pad:] = 0
            else:
                wt = weight
            trainer.step(p, t, None, wt)
    pol.refresh()
    return trainer


__all__ = ["make_training_pairs", "train_batch", "run"]

if __name__ == "__main__":
    import sys

    from ..parallel.launch import exit_status
    sys.exit(exit_status(run()))
