"""GTP time control (CPU): time_settings / time_left drive a per-move budget that the MCTS player
honours (the reference's GTP surface, interface/gtp_wrapper.py:46-65, has no clock)."""
import time

import torch

from alphago_amd import go
from alphago_amd.gtp.engine import GTPEngine
from alphago_amd.models.policy import CNNPolicy, CNNValue
from alphago_amd.search.players import MCTSPlayer

CPU = torch.device("cpu")
FEATS = ["board", "ones", "turns_since"]


def _player():
    torch.manual_seed(0)
    p = CNNPolicy(FEATS, board=19, filters_per_layer=8, layers=2, device=CPU)
    v = CNNValue(FEATS, board=19, filters_per_layer=8, layers=2, dense=16, device=CPU)
    # a playout budget no clock allows: only the time budget can end the search
    return MCTSPlayer(p, v, n_playout=10 ** 7, leaves_per_batch=8, threads=2)


def test_genmove_within_byoyomi_period():
    """time_settings 0 2 1 (2 s per move): every genmove returns inside its period, after a real search.
    (2 s rather than 1: the CPU suite runs this beside multi-process tests on a loaded host.)"""
    pl = _player()
    eng = GTPEngine(pl, size=19)
    assert eng.send("time_settings 0 2 1") == "=\n\n"
    pl.get_move(go.GameState(19), time_budget=0.05)  # warm the engines (first forwards)
    for colour in ("b", "w", "b"):
        t0 = time.perf_counter()
        reply = eng.send("genmove %s" % colour)
        dt = time.perf_counter() - t0
        assert reply.startswith("= ") and reply.strip() != "= pass", reply
        assert dt < 2.0, dt
        assert 1.5 < eng.last_budget < 2.0
    assert pl.search.forest.sims(0) > 8  # it searched, not a bare prior move


def test_clock_bookkeeping_and_time_left():
    pl = _player()
    eng = GTPEngine(pl, size=19)
    assert eng.move_budget(go.BLACK) is None  # no time settings: fixed playout budget
    eng.send("time_settings 60 10 5")  # 60 s main, then 10 s per 5 stones
    b0 = eng.move_budget(go.BLACK)
    assert 0 < b0 < 60 / 20  # main time spread over >= 20 moves
    eng.send("time_left black 4 2")  # byo-yomi: 4 s for 2 stones
    assert abs(eng.move_budget(go.BLACK) - (2.0 * 0.9 - eng.SAFETY_S)) < 1e-9
    eng.send("time_left white 0 0")  # main time used up: the byo-yomi pace
    assert eng.move_budget(go.WHITE) > 1.0
    eng.send("time_settings 0 5 0")  # byo-yomi time with 0 stones: no time limit (GTP 2)
    assert eng.move_budget(go.BLACK) is None
    eng.send("time_settings 0 1 1")
    eng._charge(go.BLACK, 0.4)  # one stone of a 1-stone period: a fresh period follows
    assert eng.clock[go.BLACK] == [1.0, 1]


def test_search_deadline_stops_inside_a_chunk():
    """BatchedMCTS.search(deadline=...): a 10^7-playout search stops at its first leaf batch past the
    deadline (the hard stop behind a loaded host's slow chunk), having searched until then."""
    pl = _player()
    st = go.GameState(19)
    pl.get_move(st, time_budget=0.05)  # warm the engines
    s0 = pl.search.forest.sims(0)
    t0 = time.perf_counter()
    pl.search.search([st], 10 ** 7, 8, 0.0, deadline=t0 + 0.3)
    assert time.perf_counter() - t0 < 1.5
    assert pl.search.forest.sims(0) > s0
