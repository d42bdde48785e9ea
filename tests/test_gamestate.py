"""Rules-engine behaviour (spec: reference tests/test_gamestate.py, test_liberties.py)."""
import numpy as np
import pytest

from alphago_amd import go


def test_standard_ko():
    gs = go.GameState(size=9)
    for m in [(1, 0), (2, 0), (0, 1), (3, 1), (1, 2), (2, 2), (2, 1)]:
        gs.do_move(m)
    gs.do_move((1, 1))  # white captures -> ko
    assert gs.num_black_prisoners == 1 and gs.num_white_prisoners == 0
    assert not gs.is_legal((2, 1))
    gs.do_move((5, 5))
    gs.do_move((5, 6))
    assert gs.is_legal((2, 1))


def test_snapback_is_not_ko():
    gs = go.GameState(size=5)
    for b, w in zip([(0, 0), (2, 1), (3, 0)], [(0, 1), (1, 1), (2, 0)]):
        gs.do_move(b)
        gs.do_move(w)
    gs.do_move((1, 0))
    assert gs.ko is None
    assert gs.is_legal((2, 0))
    gs.do_move((2, 0))
    assert gs.num_black_prisoners == 2 and gs.num_white_prisoners == 1


def test_eyeish_and_true_eye():
    gs = go.GameState(size=7)
    for m in [(1, 0), (5, 4), (2, 1), (6, 5), (1, 2), (5, 6), (0, 1), (4, 5)]:
        gs.do_move(m)
    assert gs.is_eyeish((1, 1), go.BLACK) and not gs.is_eyeish((1, 1), go.WHITE)
    assert gs.is_eyeish((5, 5), go.WHITE) and not gs.is_eyeish((5, 5), go.BLACK)
    for p in [(1, 0), (2, 2)]:
        assert not gs.is_eyeish(p, go.BLACK) and not gs.is_eyeish(p, go.WHITE)

    gs = go.GameState(size=7)
    gs.do_move((1, 0), go.BLACK)
    gs.do_move((0, 1), go.BLACK)
    assert gs.is_eyeish((0, 0), go.BLACK) and not gs.is_eye((0, 0), go.BLACK)
    for m in [(1, 2), (2, 1), (2, 2), (0, 2)]:
        gs.do_move(m, go.BLACK)
    assert gs.is_eye((0, 0), go.BLACK) and gs.is_eye((1, 1), go.BLACK)


def test_eye_recursion_checkerboard():
    gs = go.GameState(7)
    for x in range(7):
        for y in range(7):
            if (x + y) % 2 == 1:
                gs.do_move((x, y), go.BLACK)
    assert gs.is_eye((0, 0), go.BLACK)


def test_liberties_after_capture():
    cap, ref = go.GameState(7), go.GameState(7)
    for x in range(2, 5):
        for y in range(2, 5):
            cap.do_move((x, y), go.BLACK)
    for x in range(2, 5):
        for s in (cap, ref):
            s.do_move((x, 1), go.WHITE)
            s.do_move((x, 5), go.WHITE)
    for s in (cap, ref):
        s.do_move((1, 1), go.WHITE)
    for y in range(2, 5):
        for s in (cap, ref):
            s.do_move((1, y), go.WHITE)
            s.do_move((5, y), go.WHITE)
    assert np.all(ref.board == cap.board)
    assert np.all(ref.liberty_counts == cap.liberty_counts)


def test_liberty_counts_and_groups():
    s = go.GameState()
    for m in [(4, 5), (5, 5), (5, 6), (10, 10), (4, 6), (10, 11), (6, 6), (9, 10)]:
        s.do_move(m)
    assert s.liberty_counts[5][5] == 2
    assert s.liberty_counts[4][5] == 8
    assert s.liberty_counts[5][6] == 8
    st = go.GameState()
    for m in [(0, 0), (5, 5), (0, 1), (6, 6), (1, 0), (1, 1)]:
        st.do_move(m)
    assert len(st.get_group((0, 0))) == 3
    assert len(st.get_group((4, 4))) == 0
    assert len(st.get_group((5, 5))) == 1


def test_copy_has_value_semantics():
    """the reference aliases history in copy(); ours must not."""
    s = go.GameState(9, komi=6.5)
    s.do_move((2, 2))
    c = s.copy()
    c.do_move((3, 3))
    assert len(s.history) == 1 and len(c.history) == 2
    assert c.komi == 6.5


def test_illegal_moves():
    s = go.GameState(5)
    s.do_move((0, 0))
    with pytest.raises(go.IllegalMove):
        s.do_move((0, 0))
    assert not s.is_legal((-1, 0))  # Q14: bounds checked first
    assert not s.is_legal((5, 0))


def test_end_of_game_rule():
    """go.py:345-348: two consecutive passes end the game only with white to move (Q9)."""
    s = go.GameState(5)
    assert s.do_move(None) is False      # B pass
    assert s.do_move(None) is False      # W pass -> black to move: not over
    assert s.do_move(None) is True       # B pass -> white to move: over
    assert s.is_end_of_game


def test_standard_two_pass_option():
    """Q9 option: with standard_two_pass any two consecutive passes end the game;
    the flag survives copies (search slots copy leaf states)."""
    s = go.GameState(5, 7.5, standard_two_pass=True)
    assert s.standard_two_pass
    c = s.copy()
    assert c.do_move(None) is False      # B pass
    assert c.do_move(None) is True       # W pass -> over (reference rule would continue)
    assert c.is_end_of_game
    d = go.GameState(5)
    assert not d.standard_two_pass
    d.do_move((1, 1))
    d.standard_two_pass = True
    assert d.do_move(None) is False      # W pass
    assert d.do_move((2, 2)) is False    # B move resets the pass streak
    assert d.do_move(None) is False      # W pass
    assert d.do_move(None) is True       # B pass -> over
