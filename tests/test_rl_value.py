"""Self-play, RL policy training and value-network pipeline (small nets, 9x9)."""
import os

import numpy as np
import pytest
import torch

from alphago_amd import go
from alphago_amd.features import VALUE_FEATURES
from alphago_amd.models.policy import CNNPolicy, CNNValue
from alphago_amd.search.selfplay import BatchedSampler, play_games
from alphago_amd.train import rl, value

FEATS = ["board", "ones", "turns_since", "sensibleness"]


def _policy(device, board=9):
    return CNNPolicy(FEATS, board=board, filters_per_layer=16, layers=2, device=device)


def _run_selfplay(device):
    a, b = _policy(device), _policy(device)
    rec = play_games(BatchedSampler(a, seed=1), BatchedSampler(b, seed=2), 6, size=9, max_moves=200,
                     rng=np.random.default_rng(0))
    assert len(rec.winners) == 6 and set(rec.learner_colors) <= {1, -1}
    for planes, moves, st in zip(rec.planes, rec.moves, rec.states):
        assert planes.shape[0] == moves.shape[0]
        assert planes.shape[1:] == (a.preprocessor.output_dim, 9, 9)
        assert len(st.history) <= 200
    return rec


def test_selfplay_cpu():
    _run_selfplay(torch.device("cpu"))


def test_sampler_respects_masks():
    p = _policy(torch.device("cpu"))
    gs = go.GameState(9)
    for x in range(9):
        for y in range(9):
            if (x, y) != (0, 0):
                gs.do_move((x, y), go.BLACK)
    gs.current_player = go.BLACK
    assert BatchedSampler(p).get_move(gs) is go.PASS_MOVE  # only an own eye left


def _save_policy(tmp_path, device):
    p = _policy(device)
    j, w = str(tmp_path / "p.json"), str(tmp_path / "p.hdf5")
    p.save_model(j, w)
    return j, w


def test_rl_cli_cpu(tmp_path):
    j, w = _save_policy(tmp_path, "cpu")
    folder = str(tmp_path / "pool")
    out = rl.run([w, j, "--model_folder", folder, "--game_batch_size", "4", "--iterations", "2",
                  "--save_every", "1", "--minibatch", "64", "--max-moves", "120", "--backend", "torch"])
    assert len(out["history"]) == 2
    assert os.path.exists(os.path.join(folder, "weights.00001.hdf5"))
    assert len(out["pool"]) == 3
    # reference-compat loss path
    out2 = rl.run([w, j, "--game_batch_size", "2", "--iterations", "1", "--minibatch", "64", "--max-moves", "60",
                   "--loss", "reference"])
    assert out2["history"][0]["games"] == 2
    # stabilisers and model selection: weight decay, gradient clip, evaluation against the initial weights
    # every 2 iterations with the best snapshot kept
    folder3 = str(tmp_path / "pool3")
    out3 = rl.run([w, j, "--model_folder", folder3, "--game_batch_size", "4", "--iterations", "4",
                   "--save_every", "10", "--minibatch", "64", "--max-moves", "60", "--backend", "torch",
                   "--weight-decay", "1e-4", "--clip-grad-norm", "1.0", "--eval-every", "2", "--eval-games", "4"])
    evs = [r.get("eval_win_rate") for r in out3["history"]]
    assert evs[0] is None and evs[2] is None and evs[1] is not None and evs[3] is not None
    assert out3["best"]["iteration"] in (2, 4) and out3["best"]["eval_win_rate"] == max(evs[1], evs[3])
    assert os.path.exists(os.path.join(folder3, "best.hdf5"))


def test_reference_bce_update_matches_keras_semantics():
    """loss="reference": one SGD step per game on the mean binary CE of the
    softmax (Keras 1.0 binary_crossentropy, clipped), lr negated for a loss
    (reinforcement_policy_trainer.py:79-103), checked against a hand-written update."""
    import copy

    from alphago_amd.search.selfplay import GameRecords
    from alphago_amd.train.engine import TorchPolicyTrainer

    torch.manual_seed(1)
    pol = _policy(torch.device("cpu"))
    net_ref = copy.deepcopy(pol.model)
    lr = 0.5
    tr = TorchPolicyTrainer(pol.model, 4, lr=lr, device="cpu")  # CPU even where a GPU is present
    rng = np.random.default_rng(0)
    games = [(rng.integers(0, 2, (n, pol.preprocessor.output_dim, 9, 9), dtype=np.uint8),
              rng.integers(0, 81, n).astype(np.int32)) for n in (3, 6)]
    rec = GameRecords(planes=[g[0] for g in games], moves=[g[1] for g in games], winners=[1, 1],
                      learner_colors=[1, -1])  # game 0 won, game 1 lost
    out = rl.rl_update(tr, rec, 4, torch.device("cpu"), loss="reference")
    assert out["steps"] == 2 and out["positions"] == 9 and tr.policy_loss == "ce"
    params = [p for p in net_ref.parameters()]
    for (X, T), sign in zip(games, (1.0, -1.0)):
        prob = torch.softmax(net_ref.logits_torch(torch.from_numpy(X).float()), 1).clamp(1e-7, 1 - 1e-7)
        y = torch.nn.functional.one_hot(torch.from_numpy(T).long(), 81).float()
        loss = -(y * prob.log() + (1 - y) * (1 - prob).log()).mean(1).mean()
        grads = torch.autograd.grad(loss, params)
        with torch.no_grad():
            for p, g in zip(params, grads):
                p -= sign * lr * g
    for a, b in zip(pol.model.parameters(), net_ref.parameters()):
        assert torch.allclose(a, b, atol=1e-6), (a - b).abs().max()


def test_reinforce_sign():
    """A won game's moves become more likely, a lost game's less likely."""
    from alphago_amd.search.selfplay import GameRecords
    from alphago_amd.train.engine import TorchPolicyTrainer

    torch.manual_seed(0)
    pol = _policy(torch.device("cpu"))
    tr = TorchPolicyTrainer(pol.model, 16, lr=1.0, device="cpu")
    gs = go.GameState(9)
    planes = pol.preprocessor.states_to_uint8([gs])
    rec = GameRecords(planes=[planes, planes], moves=[np.array([40]), np.array([0])], winners=[1, 1],
                      learner_colors=[1, -1])
    p0 = torch.softmax(pol.model.logits_torch(torch.from_numpy(planes).float()), 1)[0]
    rl.rl_update(tr, rec, 16, torch.device("cpu"))
    p1 = torch.softmax(pol.model.logits_torch(torch.from_numpy(planes).float()), 1)[0]
    assert p1[40] > p0[40] and p1[0] < p0[0]


def test_reinforce_mean_baseline():
    """baseline="mean": an iteration the learner loses entirely leaves the weights where they are (the
    runaway that collapsed the lr 0.01 pool run, profiles/r6); baseline="none" pushes its moves down."""
    from alphago_amd.search.selfplay import GameRecords
    from alphago_amd.train.engine import TorchPolicyTrainer

    torch.manual_seed(0)
    pol = _policy(torch.device("cpu"))
    gs = go.GameState(9)
    planes = pol.preprocessor.states_to_uint8([gs])
    lost = GameRecords(planes=[planes, planes], moves=[np.array([40]), np.array([0])], winners=[-1, 1],
                       learner_colors=[1, -1])
    w0 = [p.detach().clone() for p in pol.model.parameters()]
    tr = TorchPolicyTrainer(pol.model, 16, lr=1.0, device="cpu")
    info = rl.rl_update(tr, lost, 16, torch.device("cpu"))
    assert info["baseline"] == -1.0 and info["grad_norm"] == 0.0
    assert all(torch.equal(a, b) for a, b in zip(w0, pol.model.parameters()))
    p0 = torch.softmax(pol.model.logits_torch(torch.from_numpy(planes).float()), 1)[0]
    rl.rl_update(tr, lost, 16, torch.device("cpu"), baseline="none")
    p1 = torch.softmax(pol.model.logits_torch(torch.from_numpy(planes).float()), 1)[0]
    assert (p1[40].log() + p1[0].log()) < (p0[40].log() + p0[0].log())  # the played moves, pushed down
    # mixed outcomes: won-game moves up, lost-game moves down around the mean
    mixed = GameRecords(planes=[planes, planes, planes], moves=[np.array([40]), np.array([0]), np.array([5])],
                        winners=[1, 1, 1], learner_colors=[1, 1, -1])
    info = rl.rl_update(tr, mixed, 16, torch.device("cpu"))
    assert abs(info["baseline"] - 1.0 / 3.0) < 1e-9
    # gradient clipping: the applied step is the clipped gradient's
    w1 = [p.detach().clone() for p in pol.model.parameters()]
    info = rl.rl_update(tr, mixed, 16, torch.device("cpu"), clip_grad_norm=1e-3)
    assert info["grad_norm"] > 1e-3 and not info["skipped"]
    step = torch.sqrt(sum(((a - b) ** 2).sum() for a, b in zip(pol.model.parameters(), w1)))
    assert abs(float(step) - 1e-3 * tr.sched.lr) / (1e-3 * tr.sched.lr) < 1e-3


def test_value_generate_and_train_cpu(tmp_path):
    cpu = torch.device("cpu")
    sl, rlp = _policy(cpu), _policy(cpu)
    planes, z = value.generate_positions(sl, rlp, 12, size=9, max_u=30, max_moves=150, seed=3,
                                         features=FEATS + ["color"])
    assert planes.shape[0] == z.shape[0] > 0 and set(np.unique(z)) <= {-1, 0, 1}
    # full CLI path with the 49-plane value features
    j, w = _save_policy(tmp_path, "cpu")
    data = str(tmp_path / "v.h5")
    n = value.generate_cli([j, j, data, "--games", "16", "--batch-games", "8", "--max-u", "20"])
    assert n > 0
    v = CNNValue(VALUE_FEATURES, board=9, filters_per_layer=8, layers=2, dense=16, device=cpu)
    vj = str(tmp_path / "v.json")
    v.save_model(vj)
    mpath = str(tmp_path / "vm.jsonl")
    meta = value.train_cli([vj, data, str(tmp_path / "vout"), "-B", "4", "-E", "2", "--backend", "torch",
                            "--metrics", mpath, "--log-every", "2"])
    assert len(meta["epochs"]) == 2
    assert os.path.exists(str(tmp_path / "vout" / "weights.00001.hdf5"))
    import json
    recs = [json.loads(line) for line in open(mpath)]
    steps = [r for r in recs if "step" in r]
    assert steps and all(r["step"] % 2 == 0 and r["positions_per_s"] > 0 and r["tflops"] > 0 for r in steps)
    assert len([r for r in recs if "step" not in r]) == 2


@pytest.mark.gpu
def test_selfplay_and_rl_gpu(tmp_path, cuda_device):
    _run_selfplay(cuda_device)
    j, w = _save_policy(tmp_path, "cuda")
    out = rl.run([w, j, "--game_batch_size", "8", "--iterations", "2", "--minibatch", "64", "--max-moves", "150",
                  "--backend", "hip"])
    assert len(out["history"]) == 2


@pytest.mark.gpu
def test_value_trainer_hip_matches_torch(cuda_device):
    import copy
    from alphago_amd.models.nets import ValueNet
    from alphago_amd.train.engine import HipValueTrainer, TorchValueTrainer

    torch.manual_seed(0)
    net = ValueNet(49, board=19, filters_per_layer=64, layers=3, dense=32)
    ref_net = copy.deepcopy(net)
    B = 6
    x = torch.randint(0, 2, (B, 49, 19, 19), dtype=torch.uint8, device=cuda_device)
    z = torch.tensor([1, -1, 1, 0, -1, 1], dtype=torch.float32, device=cuda_device)
    hip = HipValueTrainer(net, B, lr=0.01, device=cuda_device)
    ref = TorchValueTrainer(ref_net, B, lr=0.01, device=cuda_device)
    hip.compute_grads(x, z)
    ref.compute_grads(x, z)
    for name in hip.fp.names:
        a, b = hip.fp.grad_views[name], ref.fp.grad_views[name]
        cos = torch.nn.functional.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0).item()
        assert cos > 0.98, (name, cos)


def test_rl_resume_after_injected_fault_is_bit_identical(tmp_path, monkeypatch):
    """RL crash at iteration 2 + --resume ends with the same learner weights,
    opponent pool and history as an uninterrupted run (native rl_checkpoint.pt:
    weights, SGD iteration, pool, every RNG)."""
    from alphago_amd.train import checkpoint as ckpt
    from alphago_amd.utils import faults

    j, w = _save_policy(tmp_path, "cpu")

    def args(folder):
        return [w, j, "--model_folder", folder, "--game_batch_size", "3", "--iterations", "4", "--save_every", "1",
                "--minibatch", "32", "--max-moves", "60", "--backend", "torch", "--resume", "--seed", "3"]

    ref = rl.run(args(str(tmp_path / "ref")))
    marker = str(tmp_path / "fired")
    monkeypatch.setenv("ALPHAGO_AMD_FAULT", "raise@2:once=%s" % marker)
    faults.reload_from_env()
    try:
        with pytest.raises(faults.InjectedFault):
            rl.run(args(str(tmp_path / "run")))
        mid = ckpt.load(str(tmp_path / "run" / "rl_checkpoint.pt"))
        assert mid["iteration"] == 2
        got = rl.run(args(str(tmp_path / "run")))
    finally:
        monkeypatch.delenv("ALPHAGO_AMD_FAULT")
        faults.reload_from_env()
    a = ckpt.load(str(tmp_path / "ref" / "rl_checkpoint.pt"))
    b = ckpt.load(str(tmp_path / "run" / "rl_checkpoint.pt"))
    assert torch.equal(a["trainer"]["flat"], b["trainer"]["flat"])
    assert a["trainer"]["iterations"] == b["trainer"]["iterations"]
    assert [os.path.basename(p) for p in a["pool"]] == [os.path.basename(p) for p in b["pool"]]
    strip = lambda h: [{k: v for k, v in r.items() if not k.endswith("_per_s")} for r in h]  # noqa: E731
    assert strip(ref["history"]) == strip(got["history"])


def _torchrun_cli(argv, nproc=2, timeout=400):
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.pop("ALPHAGO_AMD_FAULT", None)
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % nproc,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, "-m", "alphago_amd"] + argv
    return subprocess.run(cmd, env=env, timeout=timeout, capture_output=True, text=True)


def test_value_pipeline_two_ranks_cli(tmp_path):
    """BASELINE config 5 as shipped, on 2 gloo ranks: value-generate writes one
    merged dataset (each rank's games, LZF-chunked), train-value trains DP on
    per-rank shards of it."""
    import json

    from alphago_amd.io.h5lite import H5File

    j, w = _save_policy(tmp_path, "cpu")
    data = str(tmp_path / "v.h5")
    r = _torchrun_cli(["value-generate", j, j, data, "--games", "6", "--batch-games", "6", "--max-u", "15"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert not os.path.exists(data + ".rank0") and not os.path.exists(data + ".rank1")
    with H5File(data) as f:
        n = f["states"].shape[0]
        assert f["states"].chunked and n == f["outcomes"].shape[0]
        assert 6 < n <= 12  # both ranks' games
        assert set(np.unique(f["outcomes"].read())) <= {-1, 0, 1}
    v = CNNValue(VALUE_FEATURES, board=9, filters_per_layer=8, layers=2, dense=16, device=torch.device("cpu"))
    vj = str(tmp_path / "v.json")
    v.save_model(vj)
    out = str(tmp_path / "vout")
    r = _torchrun_cli(["train-value", vj, data, out, "-B", "2", "-E", "2", "--backend", "torch",
                       "--train-val-test", "0.8", "0.2", "0.0"])
    assert r.returncode == 0, r.stderr[-3000:]
    meta = json.load(open(os.path.join(out, "metadata.json")))
    assert len(meta["epochs"]) == 2 and sum(meta["data"]["rows_per_rank"]) == int(0.8 * n) + int(0.2 * n)
    assert os.path.exists(os.path.join(out, "weights.00001.hdf5"))


def test_value_resume_after_injected_fault_is_bit_identical(tmp_path, monkeypatch):
    from alphago_amd.io.h5lite import H5Writer
    from alphago_amd.train import checkpoint as ckpt
    from alphago_amd.utils import faults

    rng = np.random.default_rng(0)
    data = str(tmp_path / "v.h5")
    with H5Writer(data) as f:
        f.create_chunked("states", rng.integers(0, 2, (150, len(VALUE_FEATURES) and 49, 9, 9), dtype=np.uint8), 64)
        f["outcomes"] = rng.choice([-1, 1], 150).astype(np.int8)
    torch.manual_seed(0)
    v = CNNValue(VALUE_FEATURES, board=9, filters_per_layer=8, layers=2, dense=16, device=torch.device("cpu"))
    vj = str(tmp_path / "v.json")
    v.save_model(vj, str(tmp_path / "v0.hdf5"))

    def args(out):
        return [vj, data, out, "-B", "8", "-E", "3", "--backend", "torch", "--checkpoint-every", "2", "--resume"]

    ref = value.train_cli(args(str(tmp_path / "ref")))
    marker = str(tmp_path / "fired")
    monkeypatch.setenv("ALPHAGO_AMD_FAULT", "raise@20:once=%s" % marker)  # epoch 1
    faults.reload_from_env()
    try:
        with pytest.raises(faults.InjectedFault):
            value.train_cli(args(str(tmp_path / "run")))
        got = value.train_cli(args(str(tmp_path / "run")))
    finally:
        monkeypatch.delenv("ALPHAGO_AMD_FAULT")
        faults.reload_from_env()
    a = ckpt.load(str(tmp_path / "ref" / "checkpoint.pt"))
    b = ckpt.load(str(tmp_path / "run" / "checkpoint.pt"))
    assert torch.equal(a["trainer"]["flat"], b["trainer"]["flat"])
    assert [e["loss"] for e in ref["epochs"]] == [e["loss"] for e in got["epochs"]]


@pytest.mark.gpu
def test_device_records_equal_host_records(cuda_device):
    """RL learner records kept on the device (the GPU featurizer's planes of the sampling forward)
    equal the host-featurised records: same sampled moves, same planes, same REINFORCE update."""
    from alphago_amd.features import DEFAULT_FEATURES
    from alphago_amd.models.policy import CNNPolicy
    from alphago_amd.search.selfplay import BatchedSampler, play_games
    from alphago_amd.train.engine import make_policy_trainer
    from alphago_amd.train.rl import rl_update

    torch.manual_seed(0)
    pol = CNNPolicy(DEFAULT_FEATURES, board=9, filters_per_layer=32, layers=3, device=cuda_device)
    recs, grads = [], []
    for dev_rec in (False, True):
        s1, s2 = BatchedSampler(pol, 1.0, seed=11), BatchedSampler(pol, 1.0, seed=12)
        r = play_games(s1, s2, 6, size=9, max_moves=80, rng=np.random.default_rng(4), device_records=dev_rec)
        assert isinstance(r.planes[0], torch.Tensor) == dev_rec
        recs.append(r)
        tr = make_policy_trainer(pol.model, 64, 0.0, 0.0, device=cuda_device)
        rl_update(tr, r, 64, cuda_device)
        grads.append(tr.fp.grad.clone())
    h, d = recs
    assert [list(m) for m in h.moves] == [list(m) for m in d.moves] and h.winners == d.winners
    for ph, pd in zip(h.planes, d.planes):
        assert np.array_equal(ph, pd.cpu().numpy())
    assert torch.equal(grads[0], grads[1])


def test_torch_adam_matches_keras_formula():
    """CPU: the autograd trainer's Adam is Keras 1.0 Adam (lr_t bias correction, eps on sqrt(v))."""
    import numpy as np

    from alphago_amd.models.nets import ValueNet
    from alphago_amd.train.engine import TorchValueTrainer

    torch.manual_seed(2)
    net = ValueNet(49, board=9, filters_per_layer=8, layers=2, dense=16)
    tr = TorchValueTrainer(net, 4, lr=0.002, device="cpu", optimizer="adam")
    p = tr.fp.flat.detach().double().numpy().copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    planes = torch.randint(0, 2, (4, 49, 9, 9), dtype=torch.uint8)
    z = torch.tensor([0.5, -0.2, 0.9, -1.0])
    for t in range(1, 4):
        tr.compute_grads(planes, z)
        g = tr.fp.grad.double().numpy().copy()
        tr.apply_update()
        m = 0.9 * m + 0.1 * g
        v = 0.999 * v + 0.001 * g * g
        lr_t = 0.002 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        p = p - lr_t * m / (np.sqrt(v) + 1e-8)
        np.testing.assert_allclose(tr.fp.flat.double().numpy(), p, rtol=1e-4, atol=1e-6)


def test_rl_two_ranks_cli(tmp_path):
    """train-rl under torchrun on 2 gloo ranks: every rank plays its own games, the REINFORCE gradient
    is all-reduced, rank 0 writes the snapshots / opponent pool, and the learner replicas stay equal."""
    import json

    j, w = _save_policy(tmp_path, "cpu")
    folder = str(tmp_path / "pool")
    metrics = str(tmp_path / "rl.jsonl")
    r = _torchrun_cli(["train-rl", w, j, "--model_folder", folder, "--game_batch_size", "2", "--iterations", "2",
                       "--save_every", "1", "--minibatch", "32", "--max-moves", "40", "--backend", "torch",
                       "--metrics", metrics])
    assert r.returncode == 0, r.stderr[-3000:]
    assert os.path.exists(os.path.join(folder, "weights.00001.hdf5"))
    recs = [json.loads(x) for x in open(metrics)]
    its = [x for x in recs if "games" in x]
    assert len(its) == 2 and all(x["games"] == 4 for x in its)  # both ranks' games counted



def test_value_pipeline_gpus_flag_without_torchrun(tmp_path):
    """`python -m alphago_amd value-generate/train-value --gpus 2` with no torchrun starts the two
    ranks itself (parallel/launch.py): the same merged dataset and per-rank shards as the torchrun form."""
    import json
    import subprocess
    import sys

    from alphago_amd.io.h5lite import H5File

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=root)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ALPHAGO_AMD_FAULT"):
        env.pop(k, None)

    def cli(argv):
        return subprocess.run([sys.executable, "-m", "alphago_amd"] + argv, env=env, timeout=400,
                              capture_output=True, text=True)

    j, w = _save_policy(tmp_path, "cpu")
    data = str(tmp_path / "v.h5")
    r = cli(["value-generate", j, j, data, "--games", "6", "--batch-games", "6", "--max-u", "15", "--gpus", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    with H5File(data) as f:
        n = f["states"].shape[0]
        assert 6 < n <= 12  # both ranks' games
    v = CNNValue(VALUE_FEATURES, board=9, filters_per_layer=8, layers=2, dense=16, device=torch.device("cpu"))
    vj = str(tmp_path / "v.json")
    v.save_model(vj)
    out = str(tmp_path / "vout")
    r = cli(["train-value", vj, data, out, "-B", "2", "-E", "1", "--backend", "torch", "--gpus", "2",
             "--train-val-test", "0.8", "0.2", "0.0"])
    assert r.returncode == 0, r.stderr[-3000:]
    meta = json.load(open(os.path.join(out, "metadata.json")))
    assert len(meta["data"]["rows_per_rank"]) == 2
    # a --backend hip request for more GPUs than are visible is refused, not run on fewer
    r = cli(["train-value", vj, data, out + "2", "--backend", "hip", "--gpus", "2"])
    assert r.returncode == 2 and "GPU(s) are visible" in r.stderr


def test_torch_trainer_rows_equals_gathered_batch():
    """The torch trainers take the same ``rows`` argument as the HIP ones (bench.py passes the pool
    and the drawn rows): identical to stepping on the gathered minibatch."""
    import copy

    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import TorchPolicyTrainer

    torch.manual_seed(2)
    B, C, npool = 4, 48, 10
    pool = torch.randint(0, 2, (npool, C, 19, 19), dtype=torch.uint8)
    ptgt = torch.randint(0, 361, (npool,), dtype=torch.int32)
    net = PolicyNet(C, filters_per_layer=16, layers=2)
    a = TorchPolicyTrainer(copy.deepcopy(net), B, lr=0.01, device="cpu")
    b = TorchPolicyTrainer(copy.deepcopy(net), B, lr=0.01, device="cpu")
    idx = torch.tensor([3, 3, 9, 0])
    sym = torch.tensor([0, 5, 2, 7], dtype=torch.int32)
    la = a.step(pool, ptgt.index_select(0, idx), sym, rows=idx)
    lb = b.step(pool.index_select(0, idx), ptgt.index_select(0, idx), sym)
    assert torch.equal(la[0], lb[0]) and torch.equal(a.fp.flat, b.fp.flat)
