"""Native lock-step game driver (``_engine.Lockstep``, search/lockstep.py): rules, encoding and
featurisation equal the per-state engine; on the GPU the pipelined driver plays exactly the games of
the round-3 Python loop (reference make_training_pairs, reinforcement_policy_trainer.py:16-76)."""
import numpy as np
import pytest
import torch

from alphago_amd import go
from alphago_amd._native import engine


def _random_game_pair(n_games=12, size=9, moves=60, seed=0):
    E = engine()
    rng = np.random.default_rng(seed)
    ls = E.Lockstep(n_games, size, 7.5, False, 4)
    ref = [go.GameState(size) for _ in range(n_games)]
    for _ in range(moves):
        idx = np.flatnonzero(ls.active()).astype(np.int32)
        if len(idx) == 0:
            break
        mv = []
        for i in idx:
            legal = ref[i].get_legal_moves(include_eyes=False)
            m = legal[rng.integers(len(legal))] if legal and rng.random() > 0.03 else go.PASS_MOVE
            mv.append(-1 if m is go.PASS_MOVE else m[0] * size + m[1])
            ref[i].do_move(m)
        ls.play(idx, np.asarray(mv, np.int64))
    return ls, ref


def test_lockstep_rules_match_gamestate():
    ls, ref = _random_game_pair()
    assert list(ls.active()) == [0 if s.is_end_of_game else 1 for s in ref]
    assert list(ls.to_move()) == [s.current_player for s in ref]
    assert list(ls.winners()) == [s.get_winner() for s in ref]
    assert list(ls.lengths()) == [len(s.history) for s in ref]
    for i, s in enumerate(ref):
        assert np.array_equal(ls.state(i).board_array(), s.board_array())


def test_lockstep_encode_and_featurize_match_batch_calls():
    ls, ref = _random_game_pair(seed=3)
    E = engine()
    idx = np.asarray([0, 3, 4, 7, 11], np.int32)
    k, np_ = len(idx), 81
    board = np.zeros((k + 2, np_), np.int8)
    ages = np.zeros((k + 2, np_), np.uint8)
    meta = np.zeros((k + 2, 2), np.int32)
    lad = np.zeros((k + 2, np_), np.uint8)
    ls.encode(idx, board, ages, meta, lad)
    b, a, m, l = E.encode_batch([ref[i] for i in idx], True, 2)
    assert np.array_equal(board[:k], b) and np.array_equal(ages[:k], a)
    assert np.array_equal(meta[:k], m) and np.array_equal(lad[:k], l)
    names = ["board", "ones", "turns_since", "liberties", "sensibleness", "color"]
    assert np.array_equal(ls.featurize(idx, names), E.featurize_batch([ref[i] for i in idx], names, 2))
    with pytest.raises(IndexError):
        ls.encode(np.asarray([99], np.int32), board, ages, meta, None)
    with pytest.raises(ValueError):
        ls.encode(idx, board[:2], ages, meta, None)  # buffer too small


def test_lockstep_groups_and_random_moves():
    E = engine()
    ls = E.Lockstep(6, 9, 7.5, False, 2)
    colors = np.asarray([1, -1, 1, -1, 1, 1], np.int8)
    a, b = ls.groups(colors)
    assert list(a) == [0, 2, 4, 5] and list(b) == [1, 3]
    mv = ls.play_random(np.arange(6, dtype=np.int32), 7)
    assert (mv >= 0).all() and list(ls.to_move()) == [-1] * 6
    a, b = ls.groups(colors)
    assert list(a) == [1, 3] and list(b) == [0, 2, 4, 5]
    again = E.Lockstep(6, 9, 7.5, False, 2)
    assert np.array_equal(again.play_random(np.arange(6, dtype=np.int32), 7), mv)  # seeded


@pytest.mark.gpu
@pytest.mark.parametrize("device_records", [True, False])
def test_native_driver_plays_the_python_loops_games(cuda_device, device_records):
    """Same samplers and seeds: the pipelined native driver and the Python loop sample the same moves
    (each sampler sees the same sequence of batches), so games, winners and learner records match."""
    from alphago_amd.features import DEFAULT_FEATURES
    from alphago_amd.models.policy import CNNPolicy
    from alphago_amd.search.selfplay import BatchedSampler, play_games

    torch.manual_seed(0)
    pol = CNNPolicy(DEFAULT_FEATURES, board=9, filters_per_layer=32, layers=3, device=cuda_device)
    opp = CNNPolicy(DEFAULT_FEATURES, board=9, filters_per_layer=32, layers=3, device=cuda_device)
    recs = []
    for native in (False, True):
        s1, s2 = BatchedSampler(pol, 1.0, seed=11), BatchedSampler(opp, 1.0, seed=12)
        recs.append(play_games(s1, s2, 10, size=9, max_moves=90, rng=np.random.default_rng(4),
                               device_records=device_records, native=native))
    py, nat = recs
    assert py.winners == nat.winners and py.lengths == nat.lengths and py.learner_colors == nat.learner_colors
    assert [list(m) for m in py.moves] == [list(m) for m in nat.moves]
    for a, b in zip(py.planes, nat.planes):
        a = a.cpu().numpy() if isinstance(a, torch.Tensor) else a
        b = b.cpu().numpy() if isinstance(b, torch.Tensor) else b
        assert np.array_equal(a, b)
    for a, b in zip(py.states, nat.states):
        assert np.array_equal(a.board_array(), b.board_array())


@pytest.mark.gpu
def test_native_value_generation(cuda_device):
    """Value positions on the native driver: one position per game that reached its random ply, the
    state after the random move, outcome from the recorded player's view; the 49 value planes."""
    from alphago_amd.features import DEFAULT_FEATURES
    from alphago_amd.models.policy import CNNPolicy
    from alphago_amd.train.value import VALUE_FEATURES, generate_positions

    torch.manual_seed(1)
    sl = CNNPolicy(DEFAULT_FEATURES, board=9, filters_per_layer=32, layers=3, device=cuda_device)
    rl = CNNPolicy(DEFAULT_FEATURES, board=9, filters_per_layer=32, layers=3, device=cuda_device)
    planes, z = generate_positions(sl, rl, 24, size=9, max_u=30, max_moves=120, seed=5)
    assert planes.shape[1:] == (49, 9, 9) and len(planes) == len(z) and 0 < len(z) <= 24
    assert set(np.unique(z).tolist()) <= {-1, 0, 1}
    assert len(VALUE_FEATURES) > 0
    # the "color" plane (last of the value features) is the recorded player's colour: constant per board
    col = planes[:, -1].reshape(len(planes), -1)
    assert ((col == col[:, :1]).all(1)).all()
