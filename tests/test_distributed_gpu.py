"""HIP trainer data parallelism rehearsal on one GPU: 2 ranks share cuda:0 and
exchange gradients with gloo (RCCL needs one GPU per rank; the bucketed async
all-reduce code path is the same)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, F=64, L=3, NB=16):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", ALPHAGO_AMD_DIST_BACKEND="gloo")
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.parallel import dist as agdist
    from alphago_amd.train.engine import HipPolicyTrainer

    env = agdist.init_from_env()
    dev = env.device
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=F, layers=L)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (NB, 48, 19, 19), dtype=torch.uint8, generator=g)
    tgt = torch.randint(0, 361, (NB,), dtype=torch.int32, generator=g)
    B = NB // world
    tr = HipPolicyTrainer(net, B, lr=0.1, device=dev, bucket_mb=0.05 if F == 64 else 2.0)
    sl = slice(rank * B, (rank + 1) * B)
    tr.compute_grads(planes[sl].to(dev), tgt[sl].to(dev))
    torch.cuda.synchronize()
    grad = tr.fp.grad.cpu().clone()
    tr.apply_update()
    torch.cuda.synchronize()
    # numpy copies travel by value (a shared torch tensor dies with the worker's file descriptor)
    q.put((rank, grad.numpy().copy(), len(tr.buckets), tr.fp.flat.cpu().numpy().copy()))
    agdist.barrier()
    agdist.shutdown()


@pytest.mark.parametrize("F,L,NB", [(64, 3, 16), (192, 12, 32)])
def test_hip_dp_matches_single(cuda_device, monkeypatch, F, L, NB):
    """2-rank DP (bucketed async all-reduce launched from the wgrad stream) ==
    one process on the union batch: gradients and the weights after the SGD
    step, on a small net and on the full 12-layer 192-filter benchmark net.  The weight-stationary
    forward / dgrad (B <= 16 per rank, not at the union batch) is off on both sides: its fp32 partial
    sums round to bf16 differently from the 32-pixel tile, which moves a 12-layer gradient to a cosine of
    ~0.99 -- a kernel difference, not a DP one (its own equality test: test_hip_trainer.py)."""
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    monkeypatch.setenv("ALPHAGO_AMD_WS", "0")  # (inherited by the spawned ranks)

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, F, L, NB)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    res = [(r, torch.from_numpy(g), nb, torch.from_numpy(w)) for r, g, nb, w in res]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][2] > 1  # several buckets exercised
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=F, layers=L)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (NB, 48, 19, 19), dtype=torch.uint8, generator=g)
    tgt = torch.randint(0, 361, (NB,), dtype=torch.int32, generator=g)
    tr = HipPolicyTrainer(net, NB, lr=0.1, device=cuda_device)
    tr.compute_grads(planes.to(cuda_device), tgt.to(cuda_device))
    ref = tr.fp.grad.cpu().clone()
    tr.apply_update()
    ref_w = tr.fp.flat.cpu()
    for _, grad, _, w in res:
        cos = torch.nn.functional.cosine_similarity(grad.double(), ref.double(), dim=0).item()
        assert cos > 0.9999
        assert torch.allclose(grad, ref, rtol=5e-3, atol=1e-5)
        assert torch.allclose(w, ref_w, rtol=1e-4, atol=1e-6)
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][3], res[1][3])  # replicas identical


def _rccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      ALPHAGO_AMD_FORCE_DIST="1")
    os.environ.pop("ALPHAGO_AMD_DIST_BACKEND", None)
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.parallel import dist as agdist
    from alphago_amd.train.engine import HipPolicyTrainer

    env = agdist.init_from_env()
    assert env.backend == "nccl" and env.distributed
    dev = env.device
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    g = torch.Generator().manual_seed(5)
    tr = HipPolicyTrainer(net, 32, lr=0.1, device=dev, bucket_mb=2.0)
    tr.comm_events = []
    for _ in range(3):
        planes = torch.randint(0, 2, (32, 48, 19, 19), dtype=torch.uint8, generator=g).to(dev)
        tgt = torch.randint(0, 361, (32,), dtype=torch.int32, generator=g).to(dev)
        tr.step(planes, tgt)
    stats = torch.ones(2, device=dev, dtype=torch.float64)
    agdist.all_reduce_sum_(stats)
    mx = agdist.all_reduce_max(3.5)
    agdist.barrier()
    torch.cuda.synchronize()
    q.put((tr.fp.flat.cpu().numpy().copy(), len(tr.buckets), len(tr.comm_events), float(stats.sum()), mx))
    agdist.shutdown()


def test_rccl_path_world1_matches_local(cuda_device):
    """The data-parallel collectives on RCCL itself (nccl backend, forced process group at
    world 1 -- RCCL needs one GPU per rank): parameter broadcast, bucketed async all-reduce
    during the backward, barrier and metric reductions run, and the weights equal the
    non-distributed trainer's bit for bit (a 1-rank sum is the identity)."""
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    w, nb, nev, ssum, mx = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert nb > 1 and nev == 3 and ssum == 2.0 and mx == 3.5
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    g = torch.Generator().manual_seed(5)
    tr = HipPolicyTrainer(net, 32, lr=0.1, device=cuda_device, bucket_mb=2.0)
    for _ in range(3):
        planes = torch.randint(0, 2, (32, 48, 19, 19), dtype=torch.uint8, generator=g).to(cuda_device)
        tgt = torch.randint(0, 361, (32,), dtype=torch.int32, generator=g).to(cuda_device)
        tr.step(planes, tgt)
    torch.cuda.synchronize()
    assert torch.equal(torch.from_numpy(w), tr.fp.flat.cpu())


def _rccl_graph_worker(port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      ALPHAGO_AMD_FORCE_DIST="1")
    os.environ.pop("ALPHAGO_AMD_DIST_BACKEND", None)
    if mode == "graph_ar":
        os.environ["ALPHAGO_AMD_GRAPH_ALLREDUCE"] = "1"
    if mode == "defer":
        os.environ["ALPHAGO_AMD_DEFER_ALLREDUCE"] = "1"
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.parallel import dist as agdist
    from alphago_amd.train.engine import HipPolicyTrainer

    env = agdist.init_from_env()
    dev = env.device
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    g = torch.Generator().manual_seed(5)
    tr = HipPolicyTrainer(net, 32, lr=0.1, device=dev, bucket_mb=2.0)
    if mode == "graph_ar":
        tr.enable_graphs()
    for _ in range(4):
        planes = torch.randint(0, 2, (32, 48, 19, 19), dtype=torch.uint8, generator=g).to(dev)
        tgt = torch.randint(0, 361, (32,), dtype=torch.int32, generator=g).to(dev)
        tr.step(planes, tgt)
    torch.cuda.synchronize()
    q.put((tr.fp.flat.cpu().numpy().copy(), len(tr._graphs or []) if mode == "graph_ar" else -1))
    agdist.shutdown()


@pytest.mark.parametrize("mode", ["graph_ar", "defer"])
def test_rccl_world1_graph_allreduce_and_defer(cuda_device, mode):
    """ALPHAGO_AMD_GRAPH_ALLREDUCE=1: the bucketed RCCL all-reduce captured inside ONE HIP graph with
    the whole step; ALPHAGO_AMD_DEFER_ALLREDUCE=1: every bucket launched after the backward.  Both
    on a forced world-1 RCCL group, bitwise equal to local training."""
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_graph_worker, args=(_free_port(), q, mode))
    p.start()
    w, ngraphs = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    if mode == "graph_ar":
        assert ngraphs == 1  # one graph: the all-reduce is inside it
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    g = torch.Generator().manual_seed(5)
    tr = HipPolicyTrainer(net, 32, lr=0.1, device=cuda_device, bucket_mb=2.0)
    for _ in range(4):
        planes = torch.randint(0, 2, (32, 48, 19, 19), dtype=torch.uint8, generator=g).to(cuda_device)
        tgt = torch.randint(0, 361, (32,), dtype=torch.int32, generator=g).to(cuda_device)
        tr.step(planes, tgt)
    torch.cuda.synchronize()
    assert torch.equal(torch.from_numpy(w), tr.fp.flat.cpu())


def test_comm_proxy_leaves_gradients_untouched(cuda_device, monkeypatch):
    """ALPHAGO_AMD_COMM_PROXY (one-GPU stand-in for the overlapped all-reduce) only reads the
    gradient: training with it, overlapped or deferred, equals training without it bit for bit."""
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    out = []
    for env in ({}, {"ALPHAGO_AMD_COMM_PROXY": "16,300,8"},
                {"ALPHAGO_AMD_COMM_PROXY": "16,300,8", "ALPHAGO_AMD_DEFER_ALLREDUCE": "1"}):
        for k in ("ALPHAGO_AMD_COMM_PROXY", "ALPHAGO_AMD_DEFER_ALLREDUCE"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        torch.manual_seed(0)
        tr = HipPolicyTrainer(PolicyNet(48, filters_per_layer=192, layers=12), 64, lr=0.1, device=cuda_device)
        assert (tr._proxy is not None) == bool(env)
        g = torch.Generator().manual_seed(9)
        tr.comm_events = []
        for _ in range(3):
            planes = torch.randint(0, 2, (64, 48, 19, 19), dtype=torch.uint8, generator=g).to(cuda_device)
            tgt = torch.randint(0, 361, (64,), dtype=torch.int32, generator=g).to(cuda_device)
            tr.step(planes, tgt)
        torch.cuda.synchronize()
        assert len(tr.comm_events) == (3 if env else 0)
        out.append(tr.fp.flat.cpu())
    assert torch.equal(out[0], out[1]) and torch.equal(out[0], out[2])


def _worker4(rank, world, port, q, opt, graph):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", ALPHAGO_AMD_DIST_BACKEND="gloo")
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.parallel import dist as agdist
    from alphago_amd.train.engine import HipPolicyTrainer

    env = agdist.init_from_env()
    dev = env.device
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    NB = 96
    B = NB // world
    tr = HipPolicyTrainer(net, B, lr=0.05 if opt == "sgd" else 3e-4, device=dev, bucket_mb=2.0, optimizer=opt)
    if graph:
        tr.enable_graphs()
    g = torch.Generator().manual_seed(5)
    sl = slice(rank * B, (rank + 1) * B)
    flats = []
    for _ in range(3):
        planes = torch.randint(0, 2, (NB, 48, 19, 19), dtype=torch.uint8, generator=g)
        tgt = torch.randint(0, 361, (NB,), dtype=torch.int32, generator=g)
        sym = torch.randint(0, 8, (NB,), dtype=torch.int32, generator=g)
        tr.step(planes[sl].to(dev), tgt[sl].to(dev), sym[sl].to(dev))
        torch.cuda.synchronize()
        flats.append(tr.fp.flat.cpu().numpy().copy())
    q.put((rank, tr.overlap, flats))
    agdist.barrier()
    agdist.shutdown()


@pytest.mark.parametrize("opt,graph", [("sgd", False), ("adam", False), ("sgd", True)])
def test_hip_dp_world4_auto_overlap_matches_single(cuda_device, opt, graph):
    """VERDICT r4 item 6 / ADVICE r4: 4-rank DP of the full 12 x 192 net at B = 24 per rank -- the
    automatic wgrad / dgrad stream overlap is on, the bucketed all-reduce is launched from the wgrad
    stream -- equals one process on the 96-board union batch after three steps; also with Adam (its
    moments see the reduced gradient) and with graph-captured steps (the all-reduce between the
    forward/backward and update graphs)."""
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    world, port = 4, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker4, args=(r, world, port, q, opt, graph)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res)  # the automatic overlap was on in every rank
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    tr = HipPolicyTrainer(net, 96, lr=0.05 if opt == "sgd" else 3e-4, device=cuda_device, optimizer=opt)
    w0 = tr.fp.flat.cpu().clone()
    g = torch.Generator().manual_seed(5)
    refs = []
    for _ in range(3):
        planes = torch.randint(0, 2, (96, 48, 19, 19), dtype=torch.uint8, generator=g)
        tgt = torch.randint(0, 361, (96,), dtype=torch.int32, generator=g)
        sym = torch.randint(0, 8, (96,), dtype=torch.int32, generator=g)
        tr.step(planes.to(cuda_device), tgt.to(cuda_device), sym.to(cuda_device))
        torch.cuda.synchronize()
        refs.append(tr.fp.flat.cpu().clone())
    for _, _, flats in res:
        for k, (w, ref) in enumerate(zip(flats, refs)):
            w = torch.from_numpy(w)
            # the update agrees in direction and size with the one-process update.  Per rank the B = 24
            # step runs the small-batch wgrad plan (B = 96: the per-tap plan), so the two are as close as two
            # bf16 computations of the 12-layer gradient are (each is ~0.98 cosine from fp32 autograd at
            # this init, scripts/r5/diag_small.py; test_hip_grads_match_torch uses the same 0.98); after
            # three steps the differences have been amplified through the bf16 weight rounding, and
            # Adam's per-parameter normalisation turns near-zero gradient differences into full steps
            d, dr = (w - w0).double(), (ref - w0).double()
            cos = torch.nn.functional.cosine_similarity(d, dr, dim=0).item()
            tol = 0.98 if (k == 0 and opt == "sgd") else 0.85  # Adam's first step is lr * sign(g)
            assert cos > tol and abs(d.norm().item() / dr.norm().item() - 1) < 0.05, (k, cos, d.norm(), dr.norm())
    for r in res[1:]:  # the data-parallel invariant: every replica holds the same weights at every step
        for a, b in zip(r[2], res[0][2]):
            assert (a == b).all()
