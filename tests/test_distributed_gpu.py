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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", ALPHAGO_AMD_DIST_BACKEND="gloo")
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.parallel import dist as agdist
    from alphago_amd.train.engine import HipPolicyTrainer

    env = agdist.init_from_env()
    dev = env.device
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=64, layers=3)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (16, 48, 19, 19), dtype=torch.uint8, generator=g)
    tgt = torch.randint(0, 361, (16,), dtype=torch.int32, generator=g)
    B = 16 // world
    tr = HipPolicyTrainer(net, B, lr=0.1, device=dev, bucket_mb=0.05)
    sl = slice(rank * B, (rank + 1) * B)
    tr.compute_grads(planes[sl].to(dev), tgt[sl].to(dev))
    torch.cuda.synchronize()
    q.put((rank, tr.fp.grad.cpu().clone(), len(tr.buckets)))
    agdist.barrier()
    agdist.shutdown()


def test_hip_dp_matches_single(cuda_device):
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][2] > 1  # several buckets exercised
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=64, layers=3)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (16, 48, 19, 19), dtype=torch.uint8, generator=g)
    tgt = torch.randint(0, 361, (16,), dtype=torch.int32, generator=g)
    tr = HipPolicyTrainer(net, 16, lr=0.1, device=cuda_device)
    tr.compute_grads(planes.to(cuda_device), tgt.to(cuda_device))
    ref = tr.fp.grad.cpu()
    for _, grad, _ in res:
        cos = torch.nn.functional.cosine_similarity(grad.double(), ref.double(), dim=0).item()
        assert cos > 0.9999
        assert torch.allclose(grad, ref, rtol=5e-3, atol=1e-5)
    assert torch.equal(res[0][1], res[1][1])
