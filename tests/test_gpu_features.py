"""GPU featurizer (csrc/kernels/featurize.hip) vs the CPU featurizer.

Every plane must be bit-identical to ``Preprocess`` (itself pinned to the
reference goldens in test_features.py) on random game positions, on
positions with chains of mutually-supporting eyes (the recursive is_eye
path, go.py:230-259) and on a checkerboard that overflows the kernel's
eye-frame stack (CPU fallback).
"""
import numpy as np
import pytest

from alphago_amd import go
from alphago_amd._native import engine
from alphago_amd.features import ALL_NO_LADDER_FEATURES, DEFAULT_FEATURES, VALUE_FEATURES, Preprocess


def random_positions(n, size=19, seed=0, max_len=300):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        gs = go.GameState(size)
        length = int(rng.integers(0, max_len))
        for _ in range(length):
            moves = gs.get_legal_moves(include_eyes=False)
            if not moves or rng.random() < 0.01:
                gs.do_move(go.PASS_MOVE)
            else:
                gs.do_move(moves[int(rng.integers(len(moves)))])
            if gs.is_end_of_game:
                break
        out.append(gs)
    return out


def eye_chain_positions():
    """Boards with diagonal chains of eyeish points (recursion through is_eye)."""
    res = []
    for size in (7, 9, 19):
        gs = go.GameState(size)
        # black checkerboard strip on rows 0..3 leaves diagonal eyes at odd parities
        for x in range(min(size, 6)):
            for y in range(min(size, 6)):
                if (x + y) % 2 == 1:
                    gs.do_move((x, y), go.BLACK)
        gs.do_move((size - 1, size - 1), go.WHITE)
        res.append(gs)
        gs2 = go.GameState(size)
        for x in range(size):
            for y in range(size):
                if (x + y) % 2 == 1 and x < 5:
                    gs2.do_move((x, y), go.WHITE)
        gs2.do_move((size - 1, size - 1), go.BLACK)  # white to move: white's eyes are evaluated
        res.append(gs2)
    return res


def test_encode_batch_cpu():
    states = random_positions(6, size=9, seed=3, max_len=60)
    board, ages, meta, lad = engine().encode_batch(states, False, 2)
    assert lad is None
    for i, s in enumerate(states):
        assert np.array_equal(board[i].reshape(9, 9), np.asarray(s.board))
        ts = Preprocess(["turns_since"]).state_to_uint8(s)
        exp = np.full(81, 255, np.uint8)
        for k in range(8):
            exp[ts[k].reshape(-1) == 1] = k
        assert np.array_equal(ages[i], exp)
        assert meta[i, 1] == s.current_player
    _, _, _, lad = engine().encode_batch(states, True, 2)
    assert lad.shape == (6, 81)
    for i, s in enumerate(states):
        f = Preprocess(["ladder_capture", "ladder_escape"]).state_to_uint8(s).reshape(2, -1)
        assert np.array_equal(lad[i] & 1, f[0]) and np.array_equal((lad[i] >> 1) & 1, f[1])


def test_encoded_ladders_match_planes_19x19():
    """The encoder only reads ladders at liberties of 2-liberty opponent groups
    and 1-liberty own groups; on random 19x19 games (many ataris) its bits must
    equal the ladder planes computed at every point."""
    states = random_positions(40, size=19, seed=5, max_len=250)
    _, _, _, lad = engine().encode_batch(states, True, 4)
    nz = 0
    for i, s in enumerate(states):
        f = Preprocess(["ladder_capture", "ladder_escape"]).state_to_uint8(s).reshape(2, -1)
        assert np.array_equal(lad[i] & 1, f[0]) and np.array_equal((lad[i] >> 1) & 1, f[1])
        nz += int(f.sum())
    assert nz > 0  # the sample does contain ladder moves


@pytest.mark.gpu
@pytest.mark.parametrize("feats", [ALL_NO_LADDER_FEATURES, DEFAULT_FEATURES, VALUE_FEATURES + ["legal"]])
def test_gpu_planes_match_cpu(cuda_device, feats):
    from alphago_amd.ops.gpu_features import GpuFeaturizer

    states = random_positions(48, seed=11) + eye_chain_positions()[-2:]
    fz = GpuFeaturizer(feats, board=19, device=cuda_device)
    got, sens = fz.planes(states, with_sensible=True)
    got, sens = got.cpu().numpy(), sens.cpu().numpy()
    pre = Preprocess(feats)
    for i, s in enumerate(states):
        exp = pre.state_to_uint8(s)
        if not np.array_equal(got[i], exp):
            bad = np.argwhere(got[i] != exp)
            raise AssertionError("state %d: %d mismatches, first %s" % (i, len(bad), bad[:5].tolist()))
        sm = Preprocess(["sensibleness"]).state_to_uint8(s).reshape(-1)
        assert np.array_equal(sens[i], sm)


@pytest.mark.gpu
def test_gpu_small_boards_and_eye_chains(cuda_device):
    from alphago_amd.ops.gpu_features import GpuFeaturizer

    for size in (7, 9, 19):
        states = [s for s in eye_chain_positions() if s.size == size] + random_positions(8, size, seed=size, max_len=80)
        fz = GpuFeaturizer(ALL_NO_LADDER_FEATURES + ["legal"], board=size, device=cuda_device)
        got = fz.planes(states).cpu().numpy()
        pre = Preprocess(ALL_NO_LADDER_FEATURES + ["legal"])
        for i, s in enumerate(states):
            assert np.array_equal(got[i], pre.state_to_uint8(s)), (size, i)


@pytest.mark.gpu
def test_gpu_checkerboard_overflow_fallback(cuda_device):
    import torch

    from alphago_amd.ops.gpu_features import GpuFeaturizer

    # 7x7 checkerboard: every empty point starts an eye recursion that
    # re-explores the whole diagonal lattice (exponential; ~15 ms on the CPU,
    # a 9x9 one takes ~30 s) -> the kernel's frame budget trips.
    gs = go.GameState(7)
    for x in range(7):
        for y in range(7):
            if (x + y) % 2 == 1:
                gs.do_move((x, y), go.BLACK)
    gs.do_move(go.PASS_MOVE, go.WHITE)  # black to move: every empty point is a black eye candidate
    states = [gs] + random_positions(3, size=7, seed=5, max_len=40)
    fz = GpuFeaturizer(["sensibleness", "legal"], board=7, device=cuda_device)
    board, ages, meta, lad = fz.to_device(fz.encode(states))
    ovf = torch.zeros(len(states), dtype=torch.int32, device=cuda_device)
    out = torch.empty((len(states), 2, 7, 7), dtype=torch.uint8, device=cuda_device)
    fz.run(board, ages, meta, lad, planes=out, overflow=ovf)
    assert ovf[0].item() == 1  # deep eye chain overflows the frame stack ...
    got = fz.planes(states).cpu().numpy()  # ... and is recomputed on the CPU
    pre = Preprocess(["sensibleness", "legal"])
    for i, s in enumerate(states):
        assert np.array_equal(got[i], pre.state_to_uint8(s))


@pytest.mark.gpu
def test_gpu_featurize_into_padded_input(cuda_device):
    import torch

    from alphago_amd import ops
    from alphago_amd.ops.gpu_features import GpuFeaturizer

    states = random_positions(10, seed=2)
    fz = GpuFeaturizer(DEFAULT_FEATURES, device=cuda_device)
    planes = fz.planes(states)
    ref = ops.padded_empty(len(states), 19, 2, 64, cuda_device)
    ops.pack_input(planes, ref, 2)
    board, ages, meta, lad = fz.to_device(fz.encode(states))
    out = ops.padded_empty(len(states), 19, 2, 64, cuda_device)
    sens = torch.empty((len(states), 361), dtype=torch.uint8, device=cuda_device)
    fz.run(board, ages, meta, lad, nhwc=out, P=2, sensible=sens)
    assert torch.equal(out, ref)


@pytest.mark.gpu
def test_encoded_inference_matches_planes(cuda_device):
    """evaluate_encoded (featurizer inside the graph) == evaluate(CPU planes, CPU masks)."""
    import torch

    from alphago_amd.models.policy import CNNPolicy, CNNValue

    torch.manual_seed(0)
    states = random_positions(37, seed=9)
    pol = CNNPolicy(DEFAULT_FEATURES, device=cuda_device, filters_per_layer=64, layers=3)
    eng = pol.engine
    assert eng.supports_encoded
    assert eng.needs_ladder == eng.fz.host_needs_ladder  # host ladder bits only without GPU ladders
    E = engine()
    b, a, m, l = E.encode_batch(states, True, 4)
    probs, sens, bad = eng.evaluate_encoded(b, a, m, l)
    probs, sens = probs.float().cpu().numpy().copy(), sens.cpu().numpy().copy()
    assert bad == []
    planes = Preprocess(DEFAULT_FEATURES).states_to_uint8(states)
    masks = E.featurize_batch(states, ["sensibleness"], 4).reshape(len(states), -1)
    ref = eng.evaluate(planes, masks).float().cpu().numpy()
    assert np.array_equal(sens, masks)
    np.testing.assert_array_equal(probs, ref)

    val = CNNValue(VALUE_FEATURES, device=cuda_device, filters_per_layer=64, layers=3)
    v_enc, _, _ = val.engine.evaluate_encoded(b, a, m, l)
    v_ref = val.engine.evaluate(Preprocess(VALUE_FEATURES).states_to_uint8(states))
    torch.testing.assert_close(v_enc.float().cpu(), v_ref.float().cpu())


@pytest.mark.gpu
def test_batched_mcts_encoded_path(cuda_device):
    from alphago_amd.models.policy import CNNPolicy, CNNValue
    from alphago_amd.search.mcts import BatchedMCTS

    pol = CNNPolicy(DEFAULT_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    val = CNNValue(VALUE_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    states = random_positions(4, seed=1, max_len=50)
    m = BatchedMCTS(pol, val, n_trees=4)
    assert m._encoded_engines() is not None
    moves = m.search(states, n_playout=64, leaves_per_tree=8)
    for s, mv in zip(states, moves):
        assert mv is None or s.is_legal(mv)
    # 9 trees -> two pipelined forests (5 + 4) whose GPU evaluations overlap host work
    states = random_positions(9, seed=2, max_len=60)
    mp = BatchedMCTS(pol, val, n_trees=9)
    assert len(mp._forests) == 2
    moves = mp.search(states, n_playout=48, leaves_per_tree=8)
    for i, (s, mv) in enumerate(zip(states, moves)):
        assert mv is None or s.is_legal(mv)
        assert sum(mp.forest.root_stats(i)[1]) >= 48
    mp.update_with_move(3, moves[3])
    assert np.isclose(mp.visit_distribution(0, 19).sum(), 1.0)


@pytest.mark.gpu
def test_mcts_value_side_stream_matches_serial(cuda_device, monkeypatch):
    """Small leaf batches run the value forward on a side stream beside the policy forward: the
    search statistics equal the one-stream search's."""
    from alphago_amd.models.policy import CNNPolicy, CNNValue
    from alphago_amd.search.mcts import BatchedMCTS

    pol = CNNPolicy(DEFAULT_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    val = CNNValue(VALUE_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    states = random_positions(1, seed=5, max_len=40)
    dists = []
    for flag in ("1", "0"):
        monkeypatch.setenv("ALPHAGO_AMD_MCTS_VALUE_STREAM", flag)
        m = BatchedMCTS(pol, val, n_trees=1)
        m.search(states, n_playout=96, leaves_per_tree=8)
        assert (getattr(m, "_vstream", None) is not None) == (flag == "1")
        dists.append(m.visit_distribution(0, 19))
    np.testing.assert_array_equal(dists[0], dists[1])


@pytest.mark.gpu
def test_mcts_overflow_fallback_with_two_batches_in_flight(cuda_device, monkeypatch):
    """with two leaf batches in flight and the value forward on the side stream,
    the CPU-plane fallback for overflow rows must not share bucket buffers with the batch still
    running.  Every batch reports its first row as overflowed; the search statistics equal those of
    the one-stream search with the same forced fallbacks, and the fallback used its own slot."""
    from alphago_amd.models.policy import CNNPolicy, CNNValue
    from alphago_amd.search import mcts as mcts_mod
    from alphago_amd.search.mcts import BatchedMCTS

    pol = CNNPolicy(DEFAULT_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    val = CNNValue(VALUE_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    states = random_positions(1, seed=11, max_len=60)
    dists = []
    for flag in ("1", "0"):
        monkeypatch.setenv("ALPHAGO_AMD_MCTS_VALUE_STREAM", flag)
        m = BatchedMCTS(pol, val, n_trees=1)
        for eng in (m.policy.engine, m.value.engine):
            orig = eng.collect

            def forced(handle, _orig=orig):
                out, mask, bad = _orig(handle)
                return out, mask, sorted(set(bad) | {0})

            monkeypatch.setattr(eng, "collect", forced)
        m.search(states, n_playout=160, leaves_per_tree=8)
        f = m._forests[0]
        assert f.n_pending == 0 and f.n_held == 0
        assert any(k[1] == mcts_mod.FALLBACK_SLOT for k in m.value.engine._b)
        dists.append(m.visit_distribution(0, 19))
    np.testing.assert_array_equal(dists[0], dists[1])


@pytest.mark.gpu
@pytest.mark.parametrize("leaves", [8, 32])
def test_mcts_single_tree_two_batches_in_flight(cuda_device, monkeypatch, leaves):
    """The single-tree search keeps two leaf batches in flight (Forest.hold / swap_held): it spends
    the playout budget (the held batch counts toward it: at most one batch over), leaves nothing pending or held, picks a legal
    move, and drains again on a second search of the reused tree -- with and without the pipeline."""
    from alphago_amd.models.policy import CNNPolicy, CNNValue
    from alphago_amd.search.mcts import BatchedMCTS

    pol = CNNPolicy(DEFAULT_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    val = CNNValue(VALUE_FEATURES, device=cuda_device, filters_per_layer=32, layers=2)
    states = random_positions(3, seed=7, max_len=80)
    for st in states:
        for flag in ("1", "0"):
            monkeypatch.setenv("ALPHAGO_AMD_MCTS_PIPELINE", flag)
            m = BatchedMCTS(pol, val, n_trees=1)
            mv = m.search([st], n_playout=200, leaves_per_tree=leaves)[0]
            f = m._forests[0]
            assert f.n_pending == 0 and f.n_held == 0
            visits = sum(m.forest.root_stats(0)[1])
            assert 199 <= visits <= 200 + leaves + 1, (flag, visits)  # the root expansion is a sim, not a child visit
            assert mv is None or st.is_legal(mv)
            # a second search on the same tree (subtree reuse path) also drains
            m.search([st], n_playout=64, leaves_per_tree=leaves)
            assert f.n_pending == 0 and f.n_held == 0


@pytest.mark.gpu
def test_gpu_planes_match_cpu_1000_positions(cuda_device):
    """>= 1,000 random 19x19 positions (every game length 0..330): every plane of
    the GPU featurizer (46 reference planes + ladders from the encoder + colour
    + legal) equals the CPU featurizer's, plus the sensible-move masks."""
    from alphago_amd.ops.gpu_features import GpuFeaturizer

    feats = DEFAULT_FEATURES + ["color", "legal"]
    states = random_positions(1000, seed=21, max_len=330) + eye_chain_positions()
    states = [s for s in states if s.size == 19]
    assert len(states) >= 1000
    fz = GpuFeaturizer(feats, board=19, device=cuda_device)
    pre = Preprocess(feats)
    exp_all = pre.states_to_uint8(states)
    sens_all = Preprocess(["sensibleness"]).states_to_uint8(states).reshape(len(states), -1)
    for k in range(0, len(states), 256):
        got, sens = fz.planes(states[k:k + 256], with_sensible=True)
        got, sens = got.cpu().numpy(), sens.cpu().numpy()
        exp = exp_all[k:k + 256]
        if not np.array_equal(got, exp):
            i = int(np.argwhere((got != exp).reshape(len(got), -1).any(1))[0][0])
            bad = np.argwhere(got[i] != exp[i])
            raise AssertionError("state %d: %d mismatches, first %s" % (k + i, len(bad), bad[:5].tolist()))
        assert np.array_equal(sens, sens_all[k:k + 256])


def test_bitboard_ladder_reader_matches_cpu_reader():
    """The bitboard ladder reader (csrc/engine/ladder_bb.h -- the code the GPU
    ladder kernel runs), executed on the host, gives exactly the CPU reader's
    ladder bits on 1000 random 19x19 positions and smaller boards."""
    for size, n, seed, max_len in ((19, 1000, 5, 330), (13, 300, 2, 150), (9, 300, 1, 100)):
        states = random_positions(n, size=size, seed=seed, max_len=max_len)
        board, _, meta, lad = engine().encode_batch(states, True, 8)
        got = engine().ladder_bits_bb(board, meta, size, 8)
        assert np.array_equal(got, lad), (size, np.argwhere(got != lad)[:5].tolist())
        if size == 19:
            assert int((lad & 1).sum()) > 0 and int((lad & 2).sum()) > 0


def test_ladder_node_budget_same_in_both_readers():
    """The node budget (a read gives up past N prey_loses / hunter_wins visits, like
    past the depth cap) has the same semantics and candidate order in the
    GameState-copy reader (featurize planes) and the bitboard reader (encoder,
    GPU kernel): they agree at every budget; a small one changes some bits."""
    E = engine()
    states = random_positions(400, size=19, seed=31, max_len=330)
    try:
        full = None
        for budget in (10 ** 9, 64, 0):
            E.set_ladder_budget(budget)
            board, _, meta, lad = E.encode_batch(states, True, 8)
            assert np.array_equal(E.ladder_bits_bb(board, meta, 19, 8), lad), budget
            # the encoder's bitboard searches vs the GameState-copy reader of the planes path
            pl = E.featurize_batch(states, ["ladder_capture", "ladder_escape"], 8).reshape(len(states), 2, -1)
            assert np.array_equal(pl[:, 0] | (pl[:, 1] << 1), lad), budget
            if budget == 10 ** 9:
                full = lad
            elif budget == 64:
                assert (lad != full).any()
            else:
                assert E.ladder_budget() == 4096
    finally:
        E.set_ladder_budget(0)


@pytest.mark.gpu
@pytest.mark.lab
def test_gpu_ladder_planes_match_cpu(cuda_device):
    """ladder_planes (csrc/kernels/ladder.hip) on >= 1000 random 19x19 positions
    and on 9x9 / 13x13 boards: bit-equal to the CPU ladder reader."""
    import torch
    from alphago_amd import ops

    for size, n, seed, max_len in ((19, 1200, 7, 330), (13, 200, 2, 150), (9, 200, 1, 100)):
        states = random_positions(n, size=size, seed=seed, max_len=max_len)
        board, _, meta, lad = engine().encode_batch(states, True, 8)
        out = torch.empty(board.shape, dtype=torch.uint8, device=cuda_device)
        ops.ladder_planes(torch.from_numpy(board).to(cuda_device), torch.from_numpy(meta).to(cuda_device), out, size)
        got = out.cpu().numpy()
        assert np.array_equal(got, lad), (size, np.argwhere(got != lad)[:5].tolist())
    # a small node budget: the device reader gives up exactly where the CPU reader does
    try:
        engine().set_ladder_budget(64)
        board, _, meta, lad = engine().encode_batch(random_positions(300, seed=31, max_len=330), True, 8)
        out = torch.empty(board.shape, dtype=torch.uint8, device=cuda_device)
        ops.ladder_planes(torch.from_numpy(board).to(cuda_device), torch.from_numpy(meta).to(cuda_device), out, 19)
        assert np.array_equal(out.cpu().numpy(), lad)
    finally:
        engine().set_ladder_budget(0)


@pytest.mark.gpu
@pytest.mark.lab
def test_gpu_featurizer_device_ladders(cuda_device):
    """GpuFeaturizer(gpu_ladders=True): ladder planes read on the device equal
    the CPU featurizer's, including the deep eye-chain positions."""
    from alphago_amd.ops.gpu_features import GpuFeaturizer

    feats = ["board", "ladder_capture", "ladder_escape", "sensibleness"]
    states = random_positions(64, seed=13, max_len=330) + eye_chain_positions()[-2:]
    states = [s for s in states if s.size == 19]
    fz = GpuFeaturizer(feats, board=19, device=cuda_device, gpu_ladders=True)
    assert not fz.host_needs_ladder
    got = fz.planes(states).cpu().numpy()
    assert np.array_equal(got, Preprocess(feats).states_to_uint8(states))
