"""Learnable synthetic SL data: random-game positions labelled by a fixed teacher policy.

No expert game records (KGS) are reachable offline, so the accuracy half of the headline
metric (top-1 move accuracy, /root/reference/AlphaGo/training/supervised_policy_trainer.py:
199-200) is measured on a teacher task: positions from random games, featurized by the
native featurizer into the reference's 48 planes (preprocessing.py:211-214), each labelled
with the greedy sensible move of a fixed random-init policy network.  A student of the same
architecture that learns the task raises its top-1 far above chance (1/~300); one that does
not learn stays at chance.

The teacher's move is the argmax of its probabilities averaged over the 8 board symmetries,
so the label is equivariant: the D4 augmentation of the training step (pack.hip) maps a
position and its label to another correctly labelled position.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .. import go
from .._native import engine as _native

# (k rotations by 90 degrees, transpose) for the 8 elements of D4 on (..., S, S) arrays
_D4 = [(k, t) for t in (False, True) for k in range(4)]


def _fwd(a: np.ndarray, k: int, t: bool) -> np.ndarray:
    if t:
        a = np.swapaxes(a, -1, -2)
    return np.rot90(a, k, axes=(-2, -1))


def _inv(a: np.ndarray, k: int, t: bool) -> np.ndarray:
    a = np.rot90(a, -k, axes=(-2, -1))
    if t:
        a = np.swapaxes(a, -1, -2)
    return a


def random_game_states(n: int, rng: np.random.Generator, size: int = 19, min_moves: int = 20,
                       max_moves: int = 300) -> List:
    """``n`` positions from random games (uniform over non-eye legal moves, 1 % passes); each
    game contributes the positions after each of its moves."""
    out: List = []
    while len(out) < n:
        gs = go.GameState(size)
        for _ in range(int(rng.integers(min_moves, max_moves))):
            moves = gs.get_legal_moves(include_eyes=False)
            if not moves or rng.random() < 0.01:
                gs.do_move(go.PASS_MOVE)
            else:
                gs.do_move(moves[int(rng.integers(len(moves)))])
            if gs.is_end_of_game:
                break
            out.append(gs.copy())
            if len(out) >= n:
                break
    return out[:n]


def teacher_labels(teacher, planes: np.ndarray, sensible: np.ndarray, batch: int = 1024,
                   symmetrize: bool = True) -> np.ndarray:
    """Flat move index per position: argmax over its sensible moves of the teacher's
    (D4-averaged) probabilities; -1 where no move is sensible."""
    n, S = planes.shape[0], planes.shape[-1]
    sens = sensible.reshape(n, S, S)
    acc = np.zeros((n, S, S), np.float64)
    for k, t in (_D4 if symmetrize else _D4[:1]):
        pl = np.ascontiguousarray(_fwd(planes, k, t))
        sm = np.ascontiguousarray(_fwd(sens, k, t)).reshape(n, S * S)
        for i in range(0, n, batch):
            p = teacher.engine.evaluate(pl[i:i + batch], sm[i:i + batch])
            p = p.float().cpu().numpy() if hasattr(p, "cpu") else np.asarray(p, np.float32)
            acc[i:i + batch] += _inv(p.reshape(-1, S, S), k, t)
    acc = acc.reshape(n, S * S) * (sensible.reshape(n, S * S) > 0)
    idx = acc.argmax(1).astype(np.int32)
    idx[sensible.reshape(n, S * S).sum(1) == 0] = -1
    return idx


def teacher_pool(n: int, teacher, seed: int, chunk: int = 8192, threads: int = 16,
                 symmetrize: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """(planes (n, F, S, S) uint8, targets (n,) int32 flat move index) of ``n`` teacher-labelled
    random-game positions (positions without a sensible move are replaced by further ones).
    Built in chunks of ``chunk`` positions (a GameState copy holds ~20 KB)."""
    rng = np.random.default_rng(seed)
    S = teacher.model.board
    F = teacher.preprocessor.output_dim
    planes = np.empty((n, F, S, S), np.uint8)
    tgt = np.empty((n,), np.int32)
    done = 0
    while done < n:
        sts = random_game_states(min(chunk, n - done), rng, size=S)
        pl = teacher.preprocessor.states_to_uint8(sts)
        sens = np.asarray(_native().featurize_batch(sts, ["sensibleness"], threads)).reshape(len(sts), S * S)
        lab = teacher_labels(teacher, pl, sens, symmetrize=symmetrize)
        keep = np.nonzero(lab >= 0)[0][:n - done]
        planes[done:done + len(keep)] = pl[keep]
        tgt[done:done + len(keep)] = lab[keep]
        done += len(keep)
    return planes, tgt


def value_teacher(planes_dim: int = 49, filters: int = 152, layers: int = 12, device=None, seed: int = 4343,
                  probe: np.ndarray = None, target_std: float = 1.0):
    """A fixed random-init value network (reference value.py:12-31 architecture) used as the value
    teacher.  A random init's pre-tanh outputs are nearly constant, so its last layer is rescaled so that
    the pre-tanh values on ``probe`` positions have mean 0 and std ``target_std``: the teacher's tanh
    outputs then spread over (-1, 1) and are a learnable regression target."""
    import torch

    from ..models.inference import make_value_inference
    from ..models.nets import ValueNet

    g = torch.random.get_rng_state()
    torch.manual_seed(seed)
    net = ValueNet(planes_dim, filters_per_layer=filters, layers=layers)
    torch.random.set_rng_state(g)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    net = net.to(dev)
    if probe is not None and len(probe):
        eng = make_value_inference(net, dev)
        with torch.no_grad():
            h = _value_pre_tanh(net, eng, probe)
            net.fc2_w.mul_(target_std / max(float(h.std()), 1e-12))
            net.fc2_b.copy_(net.fc2_b * 0 - float(h.mean()) * target_std / max(float(h.std()), 1e-12))
    return net


def _value_pre_tanh(net, eng, planes: np.ndarray):
    """Pre-tanh outputs (atanh of the engine's values, clipped) of ``planes``."""
    import torch

    v = []
    for i in range(0, len(planes), 1024):
        out = eng.evaluate(planes[i:i + 1024])
        out = out.float().cpu() if hasattr(out, "cpu") else torch.as_tensor(np.asarray(out, np.float32))
        v.append(out.clone())
    v = torch.cat(v).double().clamp(-1 + 1e-12, 1 - 1e-12)
    return torch.atanh(v)


def value_teacher_pool(n: int, teacher, seed: int, chunk: int = 8192, threads: int = 16,
                       symmetrize: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """(planes (n, 49, S, S) uint8, targets (n,) float32 in (-1, 1)): random-game positions featurised
    into the value net's 49 planes (AlphaGo/models/value.py:16; the 48 policy planes + colour), each
    labelled with the value teacher's tanh output averaged over the 8 board symmetries (so the D4
    augmentation of the training step keeps the labels consistent)."""
    import torch

    from ..features import VALUE_FEATURES, Preprocess
    from ..models.inference import make_value_inference

    rng = np.random.default_rng(seed)
    dev = next(teacher.parameters()).device
    eng = make_value_inference(teacher, dev)
    pre = Preprocess(VALUE_FEATURES)
    S = teacher.board
    planes = np.empty((n, pre.output_dim, S, S), np.uint8)
    tgt = np.empty((n,), np.float32)
    done = 0
    while done < n:
        sts = random_game_states(min(chunk, n - done), rng, size=S)
        pl = pre.states_to_uint8(sts, threads)
        acc = np.zeros(len(pl), np.float64)
        for k, t in (_D4 if symmetrize else _D4[:1]):
            sp = np.ascontiguousarray(_fwd(pl, k, t))
            for i in range(0, len(sp), 1024):
                out = eng.evaluate(sp[i:i + 1024])
                out = out.float().cpu().numpy() if hasattr(out, "cpu") else np.asarray(out, np.float32)
                acc[i:i + len(out)] += out
        acc /= 8 if symmetrize else 1
        planes[done:done + len(pl)] = pl
        tgt[done:done + len(pl)] = acc.astype(np.float32)
        done += len(pl)
    del torch
    return planes, tgt


def value_material_pool(n: int, seed: int, size: int = 19, threads: int = 16) -> Tuple[np.ndarray, np.ndarray]:
    """(planes (n, 49, S, S) uint8, targets (n,) float32 in (-1, 1)): random-game positions in the value
    net's 49 planes labelled tanh((d + 2 a) / s): d = own minus opponent stones (board planes 0 / 1), a =
    opponent minus own stones in atari (the one-liberty plane, 12, masked by colour), s = their standard
    deviation over the pool.  Symmetric under D4, so the augmentation keeps the labels; a learnable
    regression target (counts and a local product) for the value-net precision parity run."""
    from ..features import VALUE_FEATURES, Preprocess

    rng = np.random.default_rng(seed)
    pre = Preprocess(VALUE_FEATURES)
    planes = pre.states_to_uint8(random_game_states(n, rng, size=size), threads)[:n]
    own, opp, atari = (planes[:, i].astype(np.float32) for i in (0, 1, 12))
    raw = own.sum((1, 2)) - opp.sum((1, 2)) + 2.0 * ((opp * atari).sum((1, 2)) - (own * atari).sum((1, 2)))
    return planes, np.tanh(raw / max(float(raw.std()), 1e-6)).astype(np.float32)
