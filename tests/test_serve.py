"""Serving path: dynamic batcher and the HTTP/JSON position service."""
import threading

import numpy as np
import pytest
import torch

from alphago_amd.serve import BatchingEvaluator, GoService, make_server, post_json, random_positions


def _rowsum_fn(calls):
    def fn(planes, legal):
        calls.append(planes.shape[0])
        out = planes.reshape(planes.shape[0], -1).sum(1).astype(np.float64)
        if legal is not None:
            out = out + 1000 * legal.sum(1)
        return out[:, None]
    return fn


def test_batcher_results_match_and_batches_form():
    calls = []
    rng = np.random.default_rng(0)
    reqs = [rng.integers(0, 2, (int(rng.integers(1, 4)), 3, 5, 5), dtype=np.uint8) for _ in range(64)]
    out = [None] * len(reqs)
    with BatchingEvaluator(_rowsum_fn(calls), max_batch=16, max_wait_ms=20) as b:
        def worker(i0):
            for i in range(i0, len(reqs), 8):
                out[i] = b.evaluate(reqs[i])
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        st = b.stats()
    for r, o in zip(reqs, out):
        np.testing.assert_array_equal(o[:, 0], r.reshape(r.shape[0], -1).sum(1))
    assert max(calls) <= 16  # no round exceeds max_batch (all requests are <= 3 boards)
    assert st["requests"] == 64 and st["boards"] == sum(r.shape[0] for r in reqs)
    assert st["rounds"] < 64  # concurrent requests shared rounds


def test_batcher_single_board_legal_and_oversized():
    calls = []
    with BatchingEvaluator(_rowsum_fn(calls), max_batch=4, max_wait_ms=1) as b:
        x = np.ones((3, 5, 5), np.uint8)
        assert b.evaluate(x).shape == (1,)  # a (C, S, S) request returns its row without the batch axis
        lg = np.zeros(25, np.uint8)
        lg[:2] = 1
        assert b.evaluate(x, lg)[0] == 75 + 2000
        big = np.ones((10, 3, 5, 5), np.uint8)
        assert b.evaluate(big).shape == (10, 1)  # larger than max_batch: a round of its own
        assert 10 in calls
        with pytest.raises(ValueError, match="takes planes requests"):
            b.submit_items([object()])  # one payload kind per batcher


def test_batcher_pool_spreads_load_and_keeps_rows():
    """One batcher per device behind a pool: every request gets its own rows back and
    both devices take work."""
    from alphago_amd.serve import BatcherPool

    calls0, calls1 = [], []
    rng = np.random.default_rng(1)
    reqs = [rng.integers(0, 2, (1, 3, 5, 5), dtype=np.uint8) for _ in range(96)]
    out = [None] * len(reqs)
    with BatcherPool([BatchingEvaluator(_rowsum_fn(calls0), max_batch=8, max_wait_ms=10),
                      BatchingEvaluator(_rowsum_fn(calls1), max_batch=8, max_wait_ms=10)]) as pool:
        def worker(k):
            for i in range(k, len(reqs), 12):
                out[i] = pool.evaluate(reqs[i])
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(12)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        st = pool.stats()
    for r, o in zip(reqs, out):
        np.testing.assert_array_equal(o[:, 0], r.reshape(1, -1).sum(1))
    assert st["requests"] == 96 and sum(st["per_device_boards"]) == 96
    assert min(st["per_device_boards"]) > 0 and calls0 and calls1


def test_batcher_errors_reach_every_client_and_worker_survives():
    state = {"fail": True}

    def fn(planes, legal):
        if state["fail"]:
            raise RuntimeError("engine down")
        return np.zeros((planes.shape[0], 1))

    with BatchingEvaluator(fn, max_batch=8, max_wait_ms=5) as b:
        futs = [b.submit(np.zeros((1, 2, 3, 3), np.uint8)) for _ in range(3)]
        for f in futs:
            with pytest.raises(RuntimeError, match="engine down"):
                f.result(5)
        state["fail"] = False
        assert b.evaluate(np.zeros((2, 2, 3, 3), np.uint8)).shape == (2, 1)
        assert b.stats()["errors"] >= 1
    with pytest.raises(RuntimeError):
        b.submit(np.zeros((1, 2, 3, 3), np.uint8))  # closed


def test_batcher_rejects_malformed_requests_and_worker_survives():
    """a request whose planes shape or mask width differ from the batcher's is refused at
    submit; an assembly failure inside a round reaches that round's futures, not the worker."""
    calls = []
    with BatchingEvaluator(_rowsum_fn(calls), max_batch=8, max_wait_ms=5) as b:
        assert b.evaluate(np.ones((2, 2, 3, 3), np.uint8)).shape == (2, 1)
        with pytest.raises(ValueError, match="do not match"):
            b.submit(np.ones((1, 3, 3, 3), np.uint8))  # different plane count
        with pytest.raises(ValueError, match="width"):
            b.submit(np.ones((1, 2, 3, 3), np.uint8), np.ones((1, 10), np.uint8))  # S*S = 9
        assert b.evaluate(np.ones((1, 2, 3, 3), np.uint8), np.ones(9, np.uint8)).shape == (1, 1)
        assert b.stats()["errors"] == 0


def _service(device, value=True, size=9):
    from alphago_amd.models.policy import CNNPolicy, CNNValue

    torch.manual_seed(0)
    pol = CNNPolicy(["board", "ones", "turns_since", "liberties", "sensibleness"], board=size, filters_per_layer=16,
                    layers=3, device=device)
    val = (CNNValue(["board", "ones", "turns_since", "color"], board=size, filters_per_layer=16, layers=3, dense=16,
                    device=device) if value else None)
    return GoService(pol, val, max_batch=32, max_wait_ms=5)


def test_service_matches_direct_evaluation():
    svc = _service("cpu")
    try:
        for moves in random_positions(9, 6, max_moves=30, seed=1):
            st = svc.position(moves)
            direct = svc.policy.eval_state(st)
            got = svc.policy_moves(moves)["moves"]
            d = {m: p for m, p in direct}
            assert len(got) == len(d)
            for x, y, p in got:
                assert abs(d[(x, y)] - p) < 1e-6
            assert abs(svc.value_of(moves)["value"] - svc.value.eval_state(st)) < 1e-6
            mv = svc.genmove(moves)["move"]
            best = max(direct, key=lambda mp: mp[1])[0]
            assert tuple(mv) == best
    finally:
        svc.close()


def test_service_over_two_network_copies():
    """GoService over two copies of the network (one per device in production): same answers."""
    from alphago_amd.models.policy import CNNPolicy

    torch.manual_seed(0)
    pol = CNNPolicy(["board", "ones", "turns_since"], board=9, filters_per_layer=8, layers=2, device="cpu")
    j = None
    import tempfile, os
    with tempfile.TemporaryDirectory() as d:
        j = os.path.join(d, "m.json")
        w = os.path.join(d, "w.hdf5")
        pol.save_model(j, w)
        copies = [CNNPolicy.load_model(j, device="cpu", weights_file=w) for _ in range(2)]
    one = GoService(pol, None, max_batch=8, max_wait_ms=2)
    two = GoService(copies, None, max_batch=8, max_wait_ms=2)
    try:
        for moves in random_positions(9, 8, max_moves=20, seed=4):
            a, b = one.policy_moves(moves, top_k=3), two.policy_moves(moves, top_k=3)
            assert [m[:2] for m in a["moves"]] == [m[:2] for m in b["moves"]]
            for x, y in zip(a["moves"], b["moves"]):
                assert abs(x[2] - y[2]) < 1e-6
        assert "per_device_boards" in two.stats()["policy"]
    finally:
        one.close()
        two.close()


def test_position_cache_game_sessions():
    """Stateless clients send the whole move list every turn; the prefix cache extends the
    previous position instead of replaying the game, with identical answers."""
    svc = _service("cpu", value=False)
    ref = _service("cpu", value=False)
    ref.cache_size = 0
    try:
        game = random_positions(9, 1, max_moves=40, seed=3)[0]
        for i in range(len(game) + 1):
            a = svc.policy_moves(game[:i], top_k=4)
            b = ref.policy_moves(game[:i], top_k=4)
            assert a == b
            assert svc.position(game[:i]).board.tolist() == ref.position(game[:i]).board.tolist()
        assert svc.cache_hits >= len(game)
        assert ref.cache_hits == 0
    finally:
        svc.close()
        ref.close()


def test_http_endpoints_concurrent_clients():
    svc = _service("cpu")
    srv = make_server(svc, "127.0.0.1", 0)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    url = "http://127.0.0.1:%d" % srv.server_address[1]
    try:
        import urllib.request
        import json

        with urllib.request.urlopen(url + "/v1/health", timeout=10) as r:
            h = json.loads(r.read())
        assert h == {"ok": True, "board": 9, "value": True}
        positions = random_positions(9, 24, max_moves=20, seed=2)
        res = [None] * len(positions)

        def client(k):
            for i in range(k, len(positions), 6):
                res[i] = post_json(url + "/v1/policy", {"moves": positions[i], "top_k": 3})

        ts = [threading.Thread(target=client, args=(k,)) for k in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for r in res:
            assert len(r["moves"]) == 3 and r["moves"][0][2] >= r["moves"][1][2]
        g = post_json(url + "/v1/genmove", {"moves": positions[0], "temperature": 0.5})
        assert g["move"] is None or len(g["move"]) == 2
        v = post_json(url + "/v1/value", {"moves": positions[0]})
        assert -1.0 <= v["value"] <= 1.0
        import urllib.error

        with pytest.raises(urllib.error.HTTPError) as e:
            post_json(url + "/v1/policy", {"moves": [[4, 4], [4, 4]]})  # occupied point
        assert e.value.code == 400
        with pytest.raises(urllib.error.HTTPError) as e:
            post_json(url + "/v1/policy", {"moves": [[0, 0]] * 200000})  # over the body cap
        assert e.value.code == 413
        with pytest.raises(urllib.error.HTTPError) as e:
            post_json(url + "/v1/policy", {"moves": [None] * (4 * 81 + 1)})  # over the move cap
        assert e.value.code == 400
        st = svc.stats()["policy"]
        assert st["requests"] >= 24 + 1
    finally:
        srv.shutdown()
        srv.server_close()
        svc.close()


@pytest.mark.gpu
def test_batcher_on_hip_engine_matches_direct(cuda_device):
    """Dynamic batching over the HIP-graph policy engine (12 x 192): each client's rows
    equal a direct evaluation of the same boards."""
    from alphago_amd.models.inference import HipTrunkInference
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.serve import engine_eval_fn

    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    eng = HipTrunkInference(net, cuda_device, buckets=(8, 32, 64))
    rng = np.random.default_rng(0)
    reqs = [rng.integers(0, 2, (int(rng.integers(1, 3)), 48, 19, 19), dtype=np.uint8) for _ in range(40)]
    ref = [eng.evaluate(r).float().cpu().numpy() for r in reqs]
    out = [None] * len(reqs)
    go = threading.Barrier(8)
    with BatchingEvaluator(engine_eval_fn(eng), max_batch=64, max_wait_ms=20) as b:
        def worker(k):
            go.wait()  # all clients submit together: the first rounds must batch
            for i in range(k, len(reqs), 8):
                out[i] = b.evaluate(reqs[i])
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert b.stats()["rounds"] < len(reqs)
    # direct calls of 1-2 boards run the 8-board bucket on the split-K convs, batched rounds the 32 / 64
    # buckets unsplit: the fp32 sums run in another order (bf16 activations round differently at ~1e-3)
    for o, r in zip(out, ref):
        np.testing.assert_allclose(o, r, rtol=5e-3, atol=1e-6)


@pytest.mark.gpu
def test_service_gpu_featurizer_path_matches_planes_path(cuda_device):
    """GoService on the GPU: concurrent requests are encoded in one host call per round and
    featurised inside the engine's HIP graph; the answer equals the planes path with the
    sensibleness mask (the mask the GPU featurizer applies)."""
    from alphago_amd._native import engine as native
    from alphago_amd.features import DEFAULT_FEATURES
    from alphago_amd.models.policy import CNNPolicy

    torch.manual_seed(0)
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=12, device=cuda_device)
    assert pol.engine.supports_encoded
    svc = GoService(pol, None, max_batch=64, max_wait_ms=5)
    try:
        positions = random_positions(19, 24, max_moves=120, seed=5)
        got = [None] * len(positions)

        def client(k):
            for i in range(k, len(positions), 6):
                got[i] = svc.policy_moves(positions[i])

        ts = [threading.Thread(target=client, args=(k,)) for k in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert svc.stats()["policy"]["rounds"] < len(positions)
        for moves, g in zip(positions, got):
            st = svc.position(moves)
            planes = pol.preprocessor.states_to_uint8([st])
            sens = native().featurize_batch([st], ["sensibleness"], 1).reshape(1, -1)
            ref = pol.engine.evaluate(planes, sens).float().cpu().numpy()[0]
            d = dict(pol._select(ref, st.get_legal_moves(), 19))
            assert len(g["moves"]) == len(d)
            for x, y, p in g["moves"]:
                assert abs(d[(x, y)] - p) < 1e-4
    finally:
        svc.close()


def test_batcher_property_rows_and_bounds():
    """Property check (hypothesis): for any mix of request sizes and any max_batch, each
    request gets exactly its own rows back, and no round exceeds max_batch unless a single
    oversized request fills it alone."""
    from hypothesis import given, settings, strategies as st

    @settings(max_examples=25, deadline=None)
    @given(sizes=st.lists(st.integers(1, 9), min_size=1, max_size=40), mb=st.integers(1, 12))
    def check(sizes, mb):
        rounds = []

        def fn(planes, legal):
            rounds.append(planes.shape[0])
            return planes[:, 0, 0, :1].astype(np.int64) * 1000 + planes[:, 0, 0, 1:2]

        reqs = []
        for i, k in enumerate(sizes):
            p = np.zeros((k, 1, 1, 2), np.uint8)
            p[:, 0, 0, 0] = i % 250
            p[:, 0, 0, 1] = np.arange(k)
            reqs.append(p)
        with BatchingEvaluator(fn, max_batch=mb, max_wait_ms=0.5) as b:
            futs = [b.submit(p) for p in reqs]
            outs = [f.result(10) for f in futs]
        for i, (k, o) in enumerate(zip(sizes, outs)):
            assert o.shape == (k, 1)
            np.testing.assert_array_equal(o[:, 0], (i % 250) * 1000 + np.arange(k))
        for r in rounds:
            assert r <= mb or r in sizes
        assert sum(rounds) == sum(sizes)

    check()
