"""Run-to-run determinism of the HIP training engine.

Every reduction in the step has a fixed order (split-K wgrad slabs summed by
conv_wgrad_reduce_kernel in split order, fixed shuffle trees in the head
kernels, no float atomics on the gradient path), so two runs from the same
initial weights and batches must produce bit-identical parameters -- with or
without the second (wgrad) stream.  This is the property that makes the
native checkpoints resume bit-exactly (tests/test_fault_tolerance.py) and lets
a nondeterministic kernel change show up as a test failure instead of noise.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(device, overlap: bool, steps: int = 3, reduce_stream: bool = False):
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=4)
    B = 64
    tr = HipPolicyTrainer(net, B, lr=0.01, device=device, overlap=overlap, reduce_stream=reduce_stream)
    assert (tr.s_r is not None) == (reduce_stream and not overlap)
    g = torch.Generator().manual_seed(3)
    losses = []
    for _ in range(steps):
        planes = torch.randint(0, 2, (B, 48, 19, 19), dtype=torch.uint8, generator=g).to(device)
        tgt = torch.randint(0, 361, (B,), dtype=torch.int32, generator=g).to(device)
        sym = torch.randint(0, 8, (B,), dtype=torch.int32, generator=g).to(device)
        loss, _ = tr.step(planes, tgt, sym)
        losses.append(float(loss))
    torch.cuda.synchronize()
    return tr.fp.flat.detach().cpu().clone(), tr.fp.grad.detach().cpu().clone(), losses


def test_hip_training_bitwise_reproducible(cuda_device):
    p1, g1, l1 = _train(cuda_device, overlap=True)
    p2, g2, l2 = _train(cuda_device, overlap=True)
    assert l1 == l2
    assert torch.equal(g1, g2)
    assert torch.equal(p1, p2)


def test_hip_training_same_with_and_without_wgrad_stream(cuda_device):
    p1, g1, _ = _train(cuda_device, overlap=True)
    p2, g2, _ = _train(cuda_device, overlap=False)
    assert torch.equal(g1, g2)
    assert torch.equal(p1, p2)


def test_hip_training_same_with_and_without_reduce_stream(cuda_device):
    """Split-K reduce on its own stream beside the dgrad (double-buffered slabs):
    the same gradients and weights as the one-stream backward."""
    p1, g1, l1 = _train(cuda_device, overlap=False, steps=4)
    p2, g2, l2 = _train(cuda_device, overlap=False, steps=4, reduce_stream=True)
    assert l1 == l2
    assert torch.equal(g1, g2)
    assert torch.equal(p1, p2)


@pytest.mark.parametrize("B", [16, 64])
def test_graph_step_bitwise_equals_eager(cuda_device, B):
    """HIP-graph-captured training steps (pack, 12 convs, head, wgrad stream,
    SGD with the device-side Keras decay schedule, repack) produce exactly the
    weights and losses of the eager steps, step by step."""
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train.engine import HipPolicyTrainer

    def run(graph, static=False):
        torch.manual_seed(0)
        net = PolicyNet(48, filters_per_layer=192, layers=12)
        tr = HipPolicyTrainer(net, B, lr=0.003, decay=1e-3, device=cuda_device)
        if graph:
            tr.enable_graphs()
        g = torch.Generator(device=cuda_device)
        g.manual_seed(7)
        losses = []
        for _ in range(5):
            planes = torch.randint(0, 2, (B, 48, 19, 19), dtype=torch.uint8, device=cuda_device, generator=g)
            tgt = torch.randint(0, 361, (B,), dtype=torch.int32, device=cuda_device, generator=g)
            sym = torch.randint(0, 8, (B,), dtype=torch.int32, device=cuda_device, generator=g)
            if static:  # the batch written straight into the captured step's input buffers
                sp, st, ss = tr.static_inputs(planes, tgt, sym)
                sp.copy_(planes)
                st.copy_(tgt)
                ss.copy_(sym)
                planes, tgt, sym = sp, st, ss
            l, c = tr.step(planes, tgt, sym)
            losses.append((l.clone(), c.clone()))
        torch.cuda.synchronize()
        return tr.fp.flat.clone(), losses, tr.sched.iterations, tr

    fe, le, ie, _ = run(False)
    fg, lg, ig, tr = run(True)
    fs, ls_, is_, _ = run(True, static=True)
    assert tr._graphs is not None and len(tr._graphs) == 1
    assert ie == ig == is_ == 5
    assert torch.equal(fe, fg) and torch.equal(fe, fs)
    for (a, b), (c, d), (e, f) in zip(le, lg, ls_):
        assert torch.equal(a, c) and torch.equal(b, d)
        assert torch.equal(a, e) and torch.equal(b, f)
