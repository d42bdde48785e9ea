"""Featurizer goldens (spec: reference tests/test_preprocessing.py) + ladders."""
import numpy as np
import pytest

from alphago_amd import go
from alphago_amd.features import DEFAULT_FEATURES, Preprocess, num_planes


def simple_board():
    gs = go.GameState(size=7)
    for m in [(0, 0), (1, 0), (0, 1), (1, 1), (0, 2), (3, 4), (3, 3), (4, 5), (4, 2), (5, 4), (5, 3), (4, 3), (4, 4)]:
        gs.do_move(m)
    return gs


def self_atari_board():
    gs = go.GameState(size=7)
    for m in [(2, 4), (4, 4), (6, 0)]:
        gs.do_move(m, go.BLACK)
    for m in [(1, 0), (5, 0), (2, 3), (4, 3), (1, 4), (5, 4), (2, 5), (3, 5), (4, 5)]:
        gs.do_move(m, go.WHITE)
    return gs


def planes(gs, feats):
    return Preprocess(feats).state_to_tensor(gs)[0].transpose((1, 2, 0))


def test_plane_counts():
    assert num_planes(DEFAULT_FEATURES) == 48
    assert Preprocess(DEFAULT_FEATURES + ["color"]).output_dim == 49
    with pytest.raises(ValueError):
        Preprocess(["nope"])


def test_board_planes():
    gs = simple_board()
    f = planes(gs, ["board"])
    white = np.zeros((7, 7)); black = np.zeros((7, 7))
    for p in [(1, 0), (1, 1), (3, 4), (4, 5), (5, 4)]:
        white[p] = 1
    for p in [(0, 0), (0, 1), (0, 2), (3, 3), (4, 2), (4, 4), (5, 3)]:
        black[p] = 1
    assert np.all(f == np.dstack((white, black, 1 - white - black)))  # white to move


def test_turns_since():
    gs = simple_board()
    f = planes(gs, ["turns_since"])
    exp = np.zeros((7, 7, 8))
    rev = gs.history[::-1]
    for x in range(7):
        for y in range(7):
            if gs.board[x, y] != go.EMPTY:
                exp[x, y, min(rev.index((x, y)), 7)] = 1
    assert np.all(f == exp)


def test_liberties():
    f = planes(simple_board(), ["liberties"])
    exp = np.zeros((7, 7, 8))
    exp[4, 4, 0] = 1
    exp[0, 0:3, 1] = 1; exp[3, 4, 1] = 1; exp[5, 4, 1] = 1
    exp[1, 0:2, 2] = 1; exp[4, 5, 2] = 1; exp[3, 3, 2] = 1; exp[5, 3, 2] = 1
    exp[4, 2, 3] = 1
    assert np.all(f == exp)


def test_capture_size():
    gs = simple_board()
    f = planes(gs, ["capture_size"])
    exp = np.zeros((7, 7, 8))
    for (x, y) in gs.get_legal_moves():
        exp[x, y, 0] = 1
    assert np.all(f == exp)


def test_self_atari():
    f = planes(self_atari_board(), ["self_atari_size"])
    exp = np.zeros((7, 7, 8))
    exp[0, 0, 0] = 1
    exp[3, 4, 2] = 1
    assert np.all(f == exp)


def test_liberties_after():
    gs = simple_board()
    f = planes(gs, ["liberties_after"])
    exp = np.zeros((7, 7, 8))
    for (x, y) in gs.get_legal_moves():
        c = gs.copy()
        c.do_move((x, y))
        libs = c.liberty_counts[x, y]
        exp[x, y, libs - 1 if libs < 7 else 7] = 1
    assert np.all(f == exp)


def test_sensibleness_and_concat():
    gs = simple_board()
    f = planes(gs, ["board", "sensibleness", "capture_size"])
    exp = np.zeros((7, 7, 12))
    exp[:, :, 0] = gs.board == go.WHITE
    exp[:, :, 1] = gs.board == go.BLACK
    exp[:, :, 2] = gs.board == go.EMPTY
    for (x, y) in gs.get_legal_moves():
        if not gs.is_eye((x, y), go.WHITE):
            exp[x, y, 3] = 1
        exp[x, y, 4] = 1
    assert np.all(f == exp)


def _ladder_board(breaker=None):
    # white (3,3) with black at (2,3),(3,2),(4,2): black (3,4) starts a ladder
    # running diagonally to the lower-right edge of a 9x9 board.
    gs = go.GameState(size=9)
    for m in [(2, 3), (3, 2), (4, 2)]:
        gs.do_move(m, go.BLACK)
    gs.do_move((3, 3), go.WHITE)
    if breaker is not None:
        gs.do_move(breaker, go.WHITE)
    gs.current_player = go.BLACK
    return gs


def test_ladder_capture_and_escape():
    gs = _ladder_board()
    assert [m for m in gs.get_legal_moves() if gs.ladder_capture(m)] == [(3, 4)]
    for breaker in [(6, 6), (5, 6), (6, 5)]:  # a white stone on the path breaks it
        gs2 = _ladder_board(breaker)
        assert not any(gs2.ladder_capture(m) for m in gs2.get_legal_moves())
    gs3 = _ladder_board()
    gs3.do_move((3, 4))  # atari; white to move
    assert not gs3.ladder_escape((4, 3))
    gs4 = _ladder_board((6, 6))
    gs4.do_move((3, 4))
    assert gs4.ladder_escape((4, 3))
    f = Preprocess(["ladder_capture", "ladder_escape"]).state_to_uint8(gs4)
    assert f[1, 4, 3] == 1 and f[1].sum() == 1


def test_batch_featurize_matches_single():
    gs = simple_board()
    pp = Preprocess(DEFAULT_FEATURES + ["color"])
    states = [gs, self_atari_board(), go.GameState(7)]
    batch = pp.states_to_uint8(states)
    for i, s in enumerate(states):
        assert np.array_equal(batch[i], pp.state_to_uint8(s))


def _random_positions(n, size=9, seed=3):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        gs = go.GameState(size)
        for _ in range(int(rng.integers(20, 70))):
            moves = gs.get_legal_moves(include_eyes=False)
            if not moves:
                break
            gs.do_move(moves[int(rng.integers(len(moves)))])
        out.append(gs)
    return out


def test_capture_aware_liberties_after_matches_simulation():
    """liberties_after_exact / self_atari_size_exact (Q10 fix): the liberty count
    of the stone just played, checked against actually playing every legal move;
    positions without a capturing move agree with the reference planes."""
    feats = ["liberties_after_exact", "self_atari_size_exact", "liberties_after", "self_atari_size"]
    n_capture_moves = 0
    for gs in _random_positions(12):
        pl = planes(gs, feats)  # (x, y, 32)
        exact, satx, ref, sat = pl[..., 0:8], pl[..., 8:16], pl[..., 16:24], pl[..., 24:32]
        for (x, y) in gs.get_legal_moves(include_eyes=True):
            c = gs.copy()
            c.do_move((x, y))
            nl = int(c.liberty_counts[x][y])
            gsz = len(c.get_group((x, y)))
            want = np.zeros(8, np.uint8)
            want[min(nl, 8) - 1] = 1
            assert (exact[x, y] == want).all(), ((x, y), nl, exact[x, y])
            want_sa = np.zeros(8, np.uint8)
            if nl == 1:
                want_sa[min(gsz, 8) - 1] = 1
            assert (satx[x, y] == want_sa).all()
            captured = c.num_black_prisoners + c.num_white_prisoners - gs.num_black_prisoners - gs.num_white_prisoners
            if captured:
                n_capture_moves += 1
            else:
                assert (exact[x, y] == ref[x, y]).all() and (satx[x, y] == sat[x, y]).all()
    assert n_capture_moves > 0  # the positions exercise the capture path
