"""Differential test: native engine + featurizer vs the reference Python
implementation (loaded read-only as an oracle, see refshim.py) on random games."""
import random

import numpy as np
import pytest

import refshim
from alphago_amd import go
from alphago_amd.features import ALL_NO_LADDER_FEATURES, Preprocess

pytestmark = pytest.mark.skipif(not refshim.available(), reason="reference checkout not present")


def _random_game_pairs(size, n_moves, seed):
    rg = refshim.ref_go()
    rnd = random.Random(seed)
    ours, ref = go.GameState(size), rg.GameState(size)
    for _ in range(n_moves):
        legal = ref.get_legal_moves()
        if not legal or rnd.random() < 0.03:
            mv = None
        else:
            mv = rnd.choice(legal)
        ref.do_move(mv)
        ours.do_move(mv)
        if ref.is_end_of_game:
            break
        yield ours, ref


@pytest.mark.parametrize("size,seed", [(7, 0), (9, 1), (9, 2), (13, 3), (19, 4)])
def test_rules_match_reference(size, seed):
    rg = refshim.ref_go()
    n = {7: 120, 9: 200, 13: 300, 19: 350}[size]
    checked = 0
    for ours, ref in _random_game_pairs(size, n, seed):
        assert np.array_equal(ours.board, ref.board)
        assert np.array_equal(ours.liberty_counts, ref.liberty_counts)
        assert ours.ko == ref.ko
        assert ours.current_player == ref.current_player
        assert (ours.num_black_prisoners, ours.num_white_prisoners) == (ref.num_black_prisoners, ref.num_white_prisoners)
        assert ours.get_legal_moves() == ref.get_legal_moves()
        assert ours.get_winner() == ref.get_winner()
        if checked % 7 == 0:
            for x in range(size):
                for y in range(size):
                    if ref.board[x, y] == rg.EMPTY:
                        for c in (rg.BLACK, rg.WHITE):
                            assert ours.is_eye((x, y), c) == ref.is_eye((x, y), c)
        checked += 1
    assert checked > 20


@pytest.mark.parametrize("size,seed", [(9, 5), (19, 6)])
def test_features_match_reference(size, seed):
    rpp = refshim.ref_preprocessing().Preprocess(ALL_NO_LADDER_FEATURES)
    pp = Preprocess(ALL_NO_LADDER_FEATURES)
    for i, (ours, ref) in enumerate(_random_game_pairs(size, 260, seed)):
        if i % 5:
            continue
        a = pp.state_to_uint8(ours)
        b = rpp.state_to_tensor(ref)[0]
        assert a.shape == b.shape
        bad = np.argwhere(a != b)
        assert bad.size == 0, "plane mismatch at %s (move %d)" % (bad[:5], i)


def _sweep_positions(size, n_positions, seed):
    """Random games (restarted at game end) yielding (ours, ref) after every move."""
    rg = refshim.ref_go()
    rnd = random.Random(seed)
    ours, ref = go.GameState(size), rg.GameState(size)
    done = 0
    while done < n_positions:
        legal = ref.get_legal_moves()
        mv = None if (not legal or rnd.random() < 0.03) else rnd.choice(legal)
        ref.do_move(mv)
        ours.do_move(mv)
        done += 1
        yield ours, ref
        if ref.is_end_of_game or len(ref.history) > 3 * size * size:
            ours, ref = go.GameState(size), rg.GameState(size)


def test_rules_and_features_10k_positions():
    """>= 10^4 positions (random games on 9x9, 13x13 and
    19x19) -- rules state (board, liberties, ko, side to move, prisoners, legal
    moves, winner) after every move and all 46 reference feature planes of every
    position equal the reference implementation's."""
    rpp = refshim.ref_preprocessing().Preprocess(ALL_NO_LADDER_FEATURES)
    pp = Preprocess(ALL_NO_LADDER_FEATURES)
    total = 0
    for size, n, seed in ((9, 6000, 101), (13, 2500, 102), (19, 1500, 103)):
        for ours, ref in _sweep_positions(size, n, seed):
            assert np.array_equal(ours.board, ref.board)
            assert np.array_equal(ours.liberty_counts, ref.liberty_counts)
            assert ours.ko == ref.ko and ours.current_player == ref.current_player
            assert (ours.num_black_prisoners, ours.num_white_prisoners) == \
                (ref.num_black_prisoners, ref.num_white_prisoners)
            assert ours.get_legal_moves() == ref.get_legal_moves()
            assert ours.get_winner() == ref.get_winner()
            a = pp.state_to_uint8(ours)
            b = rpp.state_to_tensor(ref)[0]
            if not np.array_equal(a, b):
                bad = np.argwhere(a != b)
                raise AssertionError("size %d position %d: plane mismatch at %s" % (size, total, bad[:5].tolist()))
            total += 1
    assert total >= 10000


try:
    from hypothesis import given, settings, strategies as st

    @settings(max_examples=60, deadline=None, derandomize=True)
    @given(size=st.sampled_from([5, 7, 9]), picks=st.lists(st.integers(0, 1 << 20), min_size=1, max_size=150))
    def test_rules_property_random_move_sequences(size, picks):
        """Property test (hypothesis): any sequence of choices among the legal
        moves (pick % (n_legal + 1) == n_legal means pass) keeps the native
        engine and the reference in the same state, including captures, ko and
        the reference's end-of-game rule (Q9)."""
        rg = refshim.ref_go()
        ours, ref = go.GameState(size), rg.GameState(size)
        for p in picks:
            legal = ref.get_legal_moves()
            k = p % (len(legal) + 1)
            mv = None if k == len(legal) else legal[k]
            ref.do_move(mv)
            ours.do_move(mv)
            assert np.array_equal(ours.board, ref.board)
            assert np.array_equal(ours.liberty_counts, ref.liberty_counts)
            assert ours.ko == ref.ko and ours.is_end_of_game == ref.is_end_of_game
            assert ours.get_legal_moves() == ref.get_legal_moves()
            if ref.is_end_of_game:
                break
        assert ours.get_winner() == ref.get_winner()
except ImportError:  # pragma: no cover
    pass
