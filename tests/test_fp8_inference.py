"""fp8 (e4m3, block-scaled MFMA) inference engines vs the bf16 engines."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _planes(n, C, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 2, (n, C, 19, 19), dtype=torch.uint8, generator=g)


def test_fp8_policy_engine_matches_bf16(cuda_device):
    from alphago_amd.models.inference import HipTrunkInference
    from alphago_amd.models.nets import PolicyNet

    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=6).to(cuda_device)
    # spread the logits so the comparison is not trivially uniform
    with torch.no_grad():
        net.head_w.mul_(20.0)
    e16 = HipTrunkInference(net, cuda_device, precision="bf16")
    e8 = HipTrunkInference(net, cuda_device, precision="fp8")
    x = _planes(64, 48)
    p16 = e16.evaluate(x).float().cpu()
    p8 = e8.evaluate(x).float().cpu()
    assert e8.calibrated and all(-20 < e < 20 for e in e8.ex)
    assert torch.allclose(p8.sum(1), torch.ones(64), atol=1e-3)
    tv = 0.5 * (p8 - p16).abs().sum(1)  # total-variation distance per board
    assert tv.max().item() < 0.15, tv.max().item()
    # random-init nets have many near-tied logits: the top move is compared loosely
    assert (p8.argmax(1) == p16.argmax(1)).float().mean().item() > 0.6
    # second call replays the captured graph with the same scales
    p8b = e8.evaluate(x).float().cpu()
    assert torch.equal(p8, p8b)
    e8.recalibrate()
    assert torch.allclose(e8.evaluate(x).float().cpu(), p8, atol=0.05)


def test_fp8_value_engine_matches_bf16(cuda_device):
    from alphago_amd.models.inference import HipValueInference
    from alphago_amd.models.nets import ValueNet

    torch.manual_seed(1)
    net = ValueNet(49, filters_per_layer=192, layers=4).to(cuda_device)
    e16 = HipValueInference(net, cuda_device, precision="bf16")
    e8 = HipValueInference(net, cuda_device, precision="fp8")
    x = _planes(32, 49, seed=3)
    v16 = e16.evaluate(x).float().cpu()
    v8 = e8.evaluate(x).float().cpu()
    assert (v8 - v16).abs().max().item() < 0.05 + 0.1 * v16.abs().max().item()
