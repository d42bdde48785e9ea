"""Data parallelism on CPU with the gloo backend (multi-process, world_size 2)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from alphago_amd.parallel import dist as agdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, opt="sgd"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import TorchPolicyTrainer

    env = agdist.init_from_env(device="cpu")
    torch.manual_seed(0)
    net = PolicyNet(12, filters_per_layer=8, layers=2)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (8, 12, 19, 19), dtype=torch.uint8, generator=g)
    tgt = torch.randint(0, 361, (8,), dtype=torch.int32, generator=g)
    B = 8 // world
    tr = TorchPolicyTrainer(net, B, lr=0.1 if opt == "sgd" else 0.01, optimizer=opt, momentum=0.9)
    sl = slice(rank * B, (rank + 1) * B)
    tr.compute_grads(planes[sl], tgt[sl])
    grad = tr.fp.grad.clone()
    tr.step(planes[sl], tgt[sl])
    tr.step(planes[sl], tgt[sl])  # a second step: the optimizer state (momentum / Adam moments) is used
    # numpy copies travel by value (a torch tensor is shared through a file descriptor that dies with
    # the worker if the parent has not unpickled it yet)
    q.put((rank, grad.numpy().copy(), tr.fp.flat.numpy().copy()))
    agdist.barrier()
    agdist.shutdown()


@pytest.mark.parametrize("world,opt", [(2, "sgd"), (4, "sgd"), (2, "adam"), (4, "momentum")])
def test_dp_gradients_equal_single_process(world, opt):
    """world 2 / 4 DP (gloo all-reduce of the flat gradient) == one process on the union batch, with
    SGD and with the optimizers that keep state (Keras momentum / Adam: the state sees the reduced
    gradient, so it stays identical on every replica)."""
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import TorchPolicyTrainer

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, opt)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    res = [(r, torch.from_numpy(g), torch.from_numpy(f)) for r, g, f in res]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process on the full batch
    torch.manual_seed(0)
    net = PolicyNet(12, filters_per_layer=8, layers=2)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (8, 12, 19, 19), dtype=torch.uint8, generator=g)
    tgt = torch.randint(0, 361, (8,), dtype=torch.int32, generator=g)
    tr = TorchPolicyTrainer(net, 8, lr=0.1 if opt == "sgd" else 0.01, optimizer=opt, momentum=0.9)
    tr.compute_grads(planes, tgt)
    ref_grad = tr.fp.grad.clone()
    tr.step(planes, tgt)
    tr.step(planes, tgt)
    for rank, grad, flat in res:
        assert torch.allclose(grad, ref_grad, atol=1e-6, rtol=1e-4)
        assert torch.allclose(flat, tr.fp.flat, atol=1e-6, rtol=1e-4)
    for r in res[1:]:
        assert torch.equal(res[0][2], r[2])  # replicas identical


def test_buckets_cover_flat_buffer():
    segs = [(100, 10), (60, 40), (20, 40), (0, 20)]  # backward order, contiguous descending
    b = agdist.make_buckets(segs, bucket_bytes=200)
    covered = sorted((o, o + n) for o, n, _ in b)
    assert covered[0][0] == 0 and covered[-1][1] == 110
    for (a0, a1), (b0, b1) in zip(covered, covered[1:]):
        assert a1 == b0
    assert [i for _, _, ids in b for i in ids] == [0, 1, 2, 3]
    # the first layer (last in backward order) alone in the final bucket
    b = agdist.make_buckets(segs, bucket_bytes=1 << 20, last_alone=True)
    assert [ids for _, _, ids in b] == [[0, 1, 2], [3]] and b[-1][:2] == (0, 20)


def _sl_cli_torchrun(args, nproc, timeout=300):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("ALPHAGO_AMD_FAULT", None)
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % nproc,
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), "-m", "alphago_amd", "train-sl"] + args
    return subprocess.run(cmd, env=env, timeout=timeout, capture_output=True, text=True)


@pytest.mark.parametrize("resident", ["yes", "no"])
def test_dp_sharded_data_equals_single_process(tmp_path, resident):
    """2-rank SL on per-rank data shards (each rank loads ~N/2 rows; resident or
    host-streamed through the prefetch ring) ends with the same weights as a
    single process stepping on the union of the two shards' minibatches."""
    import json

    import numpy as np
    from test_fault_tolerance import _model
    from test_sl_training import _data
    from alphago_amd.train import checkpoint as ckpt

    data = _data(tmp_path)
    if resident == "no":
        # contiguous copy: the streamed shard keeps the exact permutation order
        # (block-shuffled order is only used for chunked files)
        from alphago_amd.io.h5lite import H5File, H5Writer
        with H5File(data) as f:
            states, actions = f["states"].read(), f["actions"].read()
        data = str(tmp_path / "contig.h5")
        with H5Writer(data) as f:
            f["states"] = states
            f["actions"] = actions
    model = _model(tmp_path, "cpu")
    common = ["--epochs", "1", "-l", "64", "--backend", "torch", "--no-symmetries", "-r", "0.05",
              "--resident", resident]
    mdp, msp = str(tmp_path / "dp.jsonl"), str(tmp_path / "sp.jsonl")
    r = _sl_cli_torchrun([model, data, str(tmp_path / "dp")] + common + ["-B", "8", "--metrics", mdp,
                                                                       "--log-every", "2"], 2)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _sl_cli_torchrun([model, data, str(tmp_path / "sp")] + common + ["-B", "16", "--metrics", msp,
                                                                       "--log-every", "2"], 1)
    assert r.returncode == 0, r.stderr[-3000:]
    # per-step records: the window loss is all-reduced over the ranks (a collective every
    # rank joins), so 2 ranks x 8 boards report the loss of the same 16-board windows
    sa = [json.loads(x) for x in open(mdp) if '"step"' in x]
    sb = [json.loads(x) for x in open(msp) if '"step"' in x]
    assert [x["step"] for x in sa] == [x["step"] for x in sb] == [2, 4]
    assert all(x["world"] == 2 for x in sa) and all(x["world"] == 1 for x in sb)
    for x, y in zip(sa, sb):
        assert np.isclose(x["loss"], y["loss"], rtol=1e-4) and x["acc"] == y["acc"]
    a = ckpt.load(str(tmp_path / "dp" / "checkpoint.pt"))["trainer"]["flat"]
    b = ckpt.load(str(tmp_path / "sp" / "checkpoint.pt"))["trainer"]["flat"]
    assert torch.allclose(a, b, atol=1e-6, rtol=1e-4)
    meta = json.load(open(str(tmp_path / "dp" / "metadata.json")))
    n = sum(meta["data"]["rows_per_rank"])
    assert len(meta["data"]["rows_per_rank"]) == 2
    for k in meta["data"]["rows_per_rank"]:
        assert abs(k - n / 2) <= 1
    assert meta["data"]["resident"] == (resident == "yes")
    sp = json.load(open(str(tmp_path / "sp" / "metadata.json")))
    assert np.isclose(meta["epochs"][0]["loss"], sp["epochs"][0]["loss"], rtol=1e-5)
