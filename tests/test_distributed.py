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


def _worker(rank, world, port, q):
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
    tr = TorchPolicyTrainer(net, B, lr=0.1)
    sl = slice(rank * B, (rank + 1) * B)
    tr.compute_grads(planes[sl], tgt[sl])
    grad = tr.fp.grad.clone()
    tr.step(planes[sl], tgt[sl])
    q.put((rank, grad, tr.fp.flat.clone()))
    agdist.barrier()
    agdist.shutdown()


def test_dp_gradients_equal_single_process():
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import TorchPolicyTrainer

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process on the full batch
    torch.manual_seed(0)
    net = PolicyNet(12, filters_per_layer=8, layers=2)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (8, 12, 19, 19), dtype=torch.uint8, generator=g)
    tgt = torch.randint(0, 361, (8,), dtype=torch.int32, generator=g)
    tr = TorchPolicyTrainer(net, 8, lr=0.1)
    tr.compute_grads(planes, tgt)
    ref_grad = tr.fp.grad.clone()
    tr.step(planes, tgt)
    for rank, grad, flat in res:
        assert torch.allclose(grad, ref_grad, atol=1e-6, rtol=1e-4)
        assert torch.allclose(flat, tr.fp.flat, atol=1e-6, rtol=1e-4)
    assert torch.equal(res[0][2], res[1][2])  # replicas identical


def test_buckets_cover_flat_buffer():
    segs = [(100, 10), (60, 40), (20, 40), (0, 20)]  # backward order, contiguous descending
    b = agdist.make_buckets(segs, bucket_bytes=200)
    covered = sorted((o, o + n) for o, n, _ in b)
    assert covered[0][0] == 0 and covered[-1][1] == 110
    for (a0, a1), (b0, b1) in zip(covered, covered[1:]):
        assert a1 == b0
    assert [i for _, _, ids in b for i in ids] == [0, 1, 2, 3]
