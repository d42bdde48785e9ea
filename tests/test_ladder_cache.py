"""Ladder cache of the MCTS encoder (Forest.leaf_encode, featurize.h LadderRecord): a leaf's ladder
reads are taken from its grandparent's or an encoded sibling's record wherever the boards agree on the
recorded read set.  Pinned bit-exact against encoding each leaf state from scratch, over searches on
ladder-rich positions, across advance() (the records follow the kept subtree) and a budget change."""
import numpy as np

from alphago_amd import go
from alphago_amd._native import engine
from tests.test_gpu_features import random_positions


def _encode(forest, L, np_):
    board = np.zeros((L, np_), np.int8)
    ages = np.zeros((L, np_), np.uint8)
    meta = np.zeros((L, 2), np.int32)
    lad = np.zeros((L, np_), np.uint8)
    n = forest.leaf_encode_into(board.ctypes.data, ages.ctypes.data, meta.ctypes.data, lad.ctypes.data, L, 4)
    assert n == L
    return board, lad


def _search(E, forest, rounds, leaves, rng, check):
    for _ in range(rounds):
        L = forest.gather(leaves)
        if L == 0:
            break
        np_ = forest.leaf_state(0).size ** 2
        board, lad = _encode(forest, L, np_)
        if check:
            states = [forest.leaf_state(i) for i in range(L)]
            _, _, _, ref = E.encode_batch(states, True, 4)
            assert np.array_equal(lad, ref)
        pri = rng.random((L, np_)).astype(np.float32) ** 4  # peaked priors: deep lines, many grandparents
        forest.apply(pri, rng.uniform(-1, 1, L).astype(np.float32))


def _ladder_positions():
    # random games are full of ataris; keep the ones whose encoding has ladder bits
    E = engine()
    cand = random_positions(60, size=19, seed=77, max_len=260)
    _, _, _, lad = E.encode_batch(cand, True, 4)
    return [s for s, l in zip(cand, lad) if l.any()][:4]


def test_ladder_cache_bit_exact_over_search():
    E = engine()
    rng = np.random.default_rng(5)
    pos = _ladder_positions()
    assert len(pos) >= 2
    for s in pos:
        f = E.Forest(1, 5.0, 0.0, 0, 1000, 3, 7, [])
        f.set_root(0, s)
        _search(E, f, 40, 16, rng, check=True)
        st = f.ladder_cache_stats()
        assert st["records"] > 0 and st["reused"] > 0, st
        # the records follow the kept subtree through advance()
        moves = [m for m in s.get_legal_moves(include_eyes=False)]
        f.advance(0, moves[0])
        _search(E, f, 10, 16, rng, check=True)


def test_ladder_cache_pipelined_and_budget_change():
    E = engine()
    rng = np.random.default_rng(9)
    s = _ladder_positions()[0]
    f = E.Forest(1, 5.0, 0.0, 0, 1000, 3, 3, [])
    f.set_root(0, s)
    _search(E, f, 12, 16, rng, check=False)
    # two batches in flight: the parked batch's records are references for the next gather's
    for _ in range(8):
        L = f.gather(16)
        if not L:
            break
        np_ = s.size ** 2
        _, lad = _encode(f, L, np_)
        _, _, _, ref = E.encode_batch([f.leaf_state(i) for i in range(L)], True, 4)
        assert np.array_equal(lad, ref)
        f.hold()
        L2 = f.gather(16)
        if L2:
            _, lad2 = _encode(f, L2, np_)
            _, _, _, ref2 = E.encode_batch([f.leaf_state(i) for i in range(L2)], True, 4)
            assert np.array_equal(lad2, ref2)
            f.apply(rng.random((L2, np_)).astype(np.float32), rng.uniform(-1, 1, L2).astype(np.float32))
        f.swap_held()
        f.apply(rng.random((L, np_)).astype(np.float32), rng.uniform(-1, 1, L).astype(np.float32))
    # a different node budget never reuses records read under the old one
    try:
        E.set_ladder_budget(64)
        _search(E, f, 6, 16, rng, check=True)
    finally:
        E.set_ladder_budget(0)
    # cache off: same planes
    f.ladder_cache = False
    assert f.ladder_cache_stats()["records"] == 0
    _search(E, f, 4, 16, rng, check=True)


def test_ladder_cache_byte_budget_evicts_instead_of_freezing():
    """The cache holds at most its byte budget (per tree: budget / trees); a full tree drops its own
    records and keeps caching (counted in 'evictions'); 'bytes' reports the host memory held."""
    E = engine()
    rng = np.random.default_rng(3)
    s = _ladder_positions()[0]
    f = E.Forest(1, 5.0, 0.0, 0, 1000, 3, 5, [])
    f.set_root(0, s)
    _search(E, f, 12, 16, rng, check=True)
    st = f.ladder_cache_stats()
    assert st["records"] > 0 and st["bytes"] > 0 and st["evictions"] == 0
    assert st["budget_bytes"] == 256 << 20
    per = st["bytes"] / st["records"]
    f.set_ladder_cache_bytes(1 << 20)  # the floor: 1 MiB
    budget = f.ladder_cache_stats()["budget_bytes"]
    assert budget == 1 << 20
    f.set_root(0, s)
    assert f.ladder_cache_stats()["bytes"] == 0
    _search(E, f, 100, 16, rng, check=True)  # planes stay exact across evictions
    st = f.ladder_cache_stats()
    assert st["bytes"] <= budget + 16 * per and st["records"] > 0
    assert st["evictions"] >= 1  # ~2 KB records: 1 MiB fills within 100 rounds of 16 leaves
