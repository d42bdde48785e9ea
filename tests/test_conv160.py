"""160-wide conv tiles (value net: 152 filters padded to 160, AlphaGo/models/value.py:7)
vs plain PyTorch fp32: forward with straddled K-steps (Cin % 64 == 32), the
ReLU'-bitmask dgrad, and the 160x160 / tap-merged 160x64 wgrad tiles."""
import math

import pytest
import torch
import torch.nn.functional as F
from _marks import lab_params

pytestmark = pytest.mark.gpu

PROD_160 = (0, 36, 64, 128, 256, 384, 385, 386, 387)


def _conv_fwd(ops, tile, x, w, bias, y, K, S, Pin, Po=1, mode=0, mbits=None):
    """Production tiles through torch.ops.alphago_amd, the LDS-ring tiles 65 / 130 (kernel lab since
    round 5) through torch.ops.alphago_amd_lab."""
    if tile in PROD_160:
        return ops.conv_fwd(x, w, bias, y, K, S, Pin, Po, mode=mode, mbits=mbits, tile=tile)
    ops.lab().conv_fwd(x, w, bias, None, y, K, S, Pin, Po, mode, mbits, tile)
    return y


@pytest.fixture(scope="module")
def ops(cuda_device):
    from alphago_amd import ops as _ops

    _ops.load()
    return _ops


def _bf(x):
    return x.to(torch.bfloat16).float()


def _rel_err(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)


def test_padding_helpers(ops):
    assert ops.pad_filters(152) == 160 and ops.pad_filters(192) == 192 and ops.pad_filters(64) == 64
    assert ops.mbits_words(160) == 8 and ops.conv_n_tile(160) == 160
    w = torch.zeros(152, 152, 3, 3)
    assert ops.packed_weight_like(w, 160, 160).shape == (10, 160, 160)  # extra zero tap
    assert ops.packed_weight_like(torch.zeros(152, 49, 5, 5), 64, 160).shape == (25, 160, 64)


@pytest.mark.parametrize("tile", lab_params([0, 36, 64, 65, 128, 130, 256, 384, 385, 386, 387], PROD_160))
@pytest.mark.parametrize("B,Cin,Cin_p,K", [(5, 152, 160, 3), (3, 49, 64, 5), (1, 152, 160, 3)])
def test_conv_fwd_160(ops, cuda_device, tile, B, Cin, Cin_p, K):
    torch.manual_seed(0)
    S, P, Cout, Cp = 19, K // 2, 152, 160
    x = _bf(torch.randn(B, Cin, S, S, device=cuda_device))
    w = _bf(torch.randn(Cout, Cin, K, K, device=cuda_device) * 0.05)
    b = torch.randn(Cout, device=cuda_device) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=P))
    xp = ops.to_padded(x, P, Cin_p)
    wp = ops.packed_weight_like(w, Cin_p, Cp)
    ops.pack_weights([w.contiguous()], [wp])
    bp = torch.zeros(Cp, device=cuda_device)
    bp[:Cout] = b
    y = ops.padded_empty(B, S, 1, Cp, cuda_device)
    mbits = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(Cp), dtype=torch.int32, device=cuda_device)
    _conv_fwd(ops, tile, xp, wp, bp, y, K, S, P, 1, mbits=mbits)
    torch.cuda.synchronize()
    out = ops.from_padded(y, 1)
    assert _rel_err(out[:, :Cout], ref) < 1e-2
    assert out[:, Cout:].abs().sum() == 0  # padded channels: zero weights, zero bias
    assert y[:, 0].abs().sum() == 0 and y[:, :, -1].abs().sum() == 0


@pytest.mark.parametrize("tile", lab_params([0, 36, 64, 65, 130, 128, 384, 385, 386, 387], PROD_160))
def test_conv_dgrad_160_bitmask(ops, cuda_device, tile):
    """dgrad with transposed 160-wide weights and the ReLU' bitmask written by
    the forward epilogue == conv2d_input * (y > 0)."""
    torch.manual_seed(1)
    B, S, K, C, Cp = 4, 19, 3, 152, 160
    xin = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w0 = _bf(torch.randn(C, C, K, K, device=cuda_device) * 0.05)
    b0 = torch.randn(C, device=cuda_device) * 0.1
    w = _bf(torch.randn(C, C, K, K, device=cuda_device) * 0.05)
    dz = _bf(torch.randn(B, C, S, S, device=cuda_device))
    # forward of the previous layer: y = relu(conv(xin, w0) + b0), bitmask written alongside
    wp0 = ops.packed_weight_like(w0, Cp, Cp)
    ops.pack_weights([w0], [wp0])
    bp0 = torch.zeros(Cp, device=cuda_device)
    bp0[:C] = b0
    y = ops.padded_empty(B, S, 1, Cp, cuda_device)
    mbits = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(Cp), dtype=torch.int32, device=cuda_device)
    _conv_fwd(ops, tile, ops.to_padded(xin, 1, Cp), wp0, bp0, y, K, S, 1, 1, mbits=mbits)
    yv = ops.from_padded(y, 1)[:, :C]
    ref = torch.nn.grad.conv2d_input((B, C, S, S), w, dz, padding=K // 2) * (yv > 0)
    wf = ops.packed_weight_like(w, Cp, Cp)
    wd = ops.packed_weight_like(w, Cp, Cp, transposed=True)
    ops.pack_weights([w], [wf], [wd])
    dx = ops.padded_empty(B, S, 1, Cp, cuda_device)
    _conv_fwd(ops, tile, ops.to_padded(dz, 1, Cp), wd, None, dx, K, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mbits)
    torch.cuda.synchronize()
    out = ops.from_padded(dx, 1)
    assert _rel_err(out[:, :C], ref) < 1e-2
    assert out[:, C:].abs().sum() == 0


@pytest.mark.parametrize("variant", [0, pytest.param(9, marks=pytest.mark.lab), pytest.param(5, marks=pytest.mark.lab)])
@pytest.mark.parametrize("B,Cin,Cin_p,K,Pin", [(6, 152, 160, 3, 1), (5, 49, 64, 5, 2), (3, 152, 160, 3, 1)])
def test_conv_wgrad_160(ops, cuda_device, B, Cin, Cin_p, K, Pin, variant):
    """variant 0: per-tap 160x160 / tap-merged 160x64 kernels; 5: the one-kernel-row wgrad."""
    torch.manual_seed(2)
    S, Cout, Cp = 19, 152, 160
    x = _bf(torch.randn(B, Cin, S, S, device=cuda_device))
    dz = _bf(torch.randn(B, Cout, S, S, device=cuda_device))
    ref_w = torch.nn.grad.conv2d_weight(x, (Cout, Cin, K, K), dz, padding=K // 2)
    ref_b = dz.sum(dim=(0, 2, 3))
    xp = ops.to_padded(x, Pin, Cin_p)
    dzp = ops.to_padded(dz, 1, Cp)
    taps = ops.wgrad_tap_group(Cp, Cin_p, K)
    assert taps == (K if Cin_p == 64 else 1)
    ns = ops.wgrad_splits(B * S * S, K * K // taps)
    slab = torch.full((ns, K * K, Cp, Cin_p), float("nan"), device=cuda_device)
    dbs = torch.zeros(ns, Cp, device=cuda_device)
    if variant != 0:  # 5: the one-kernel-row wgrad, 9: the LDS-ring wgrad (kernel lab)
        ops.lab().conv_wgrad(xp, dzp, slab, dbs, K, S, Pin, 1, Cin if Cin_p == 64 else 0, variant)
    else:
        ops.conv_wgrad(xp, dzp, slab, dbs, K, S, Pin, 1, cin_real=Cin if Cin_p == 64 else 0, variant=variant)
    gw = torch.zeros(Cout, Cin, K, K, device=cuda_device)
    gb = torch.zeros(Cout, device=cuda_device)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert _rel_err(gw, ref_w) < 2e-3
    assert _rel_err(gb, ref_b) < 2e-3


@pytest.mark.parametrize("B,Cin,Cin_p,K", [(5, 152, 160, 3), (3, 49, 64, 5)])
@pytest.mark.parametrize("cw", [32, 64])
def test_conv_fwd_fp8_160(ops, cuda_device, monkeypatch, cw, B, Cin, Cin_p, K):
    """e4m3 conv with 160-channel activations (three 64-channel chunks per tap,
    the third one's upper half reads the next pixel against zero weights) and a
    160-wide output tile vs fp32 conv of the dequantised operands."""
    monkeypatch.setenv("ALPHAGO_AMD_FP8_CW32", "1" if cw == 32 else "0")  # 160-channel packs: 32 / 64-channel chunks
    torch.manual_seed(3)
    S, P, Cout, Cp = 19, K // 2, 152, 160
    x = F.relu(torch.randn(B, Cin, S, S, device=cuda_device)) * 3.0
    w = torch.randn(Cout, Cin, K, K, device=cuda_device) * 0.05
    b = torch.randn(Cout, device=cuda_device) * 0.1
    bp = torch.zeros(Cp, device=cuda_device)
    bp[:Cout] = b
    xp = ops.to_padded(x, P, Cin_p)
    ex = ops.fp8_exponent(float(x.abs().max()), margin=0)
    x8 = torch.empty(xp.shape, dtype=torch.uint8, device=cuda_device)
    ops.quantize_fp8(xp, x8, ex)
    w8, ew = ops.pack_weights_fp8(w, Cp, Cin_p)
    assert tuple(w8.shape) == ops.fp8_weight_shape(K, Cin_p, Cp)
    xq = ops.fp8_to_float(x8, ex)[:, P:P + S, P:P + S, :Cin].permute(0, 3, 1, 2)
    wq = (w * 2.0 ** ew).clamp(-448, 448).to(torch.float8_e4m3fn).float() * 2.0 ** -ew
    ref = F.relu(F.conv2d(xq, wq, b, padding=P))
    scales = torch.tensor([127 - ex, 127 - ew], dtype=torch.int32, device=cuda_device)
    ey = ops.fp8_exponent(float(ref.max()), margin=0)
    osc = torch.tensor([2.0 ** ey], device=cuda_device)
    amax = ops.fp8_amax_buffer(1, cuda_device)[0]
    yb = ops.padded_empty(B, S, 1, Cp, cuda_device)
    y8 = torch.zeros((B, S + 2, S + 2, Cp), dtype=torch.uint8, device=cuda_device)
    mbits = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(Cp), dtype=torch.int32, device=cuda_device)
    ops.conv_fwd_fp8(x8, w8, bp, scales, osc, K, S, P, 1, y_bf16=yb, y_fp8=y8, amax=amax, mbits=mbits)
    torch.cuda.synchronize()
    out = ops.from_padded(yb, 1)
    assert _rel_err(out[:, :Cout], ref) < 1e-2
    assert out[:, Cout:].abs().sum() == 0
    assert _rel_err(ops.fp8_to_float(y8, ey)[:, 1:S + 1, 1:S + 1, :Cout].permute(0, 3, 1, 2), ref) < 0.07
    assert y8[:, 0].sum() == 0 and y8[:, :, 0].sum() == 0 and y8[:, S + 1].sum() == 0  # borders untouched
    assert abs(amax.view(torch.float32).max().item() - ref.max().item()) <= 1e-2 * ref.max().item()
    # the ReLU' bitmask written by the fp8 epilogue == masking by y_bf16 > 0 in the bf16 dgrad
    w2 = _bf(torch.randn(Cout, Cout, 3, 3, device=cuda_device) * 0.05)
    wf2 = ops.packed_weight_like(w2, Cp, Cp)
    wd2 = ops.packed_weight_like(w2, Cp, Cp, transposed=True)
    ops.pack_weights([w2], [wf2], [wd2])
    dz = ops.to_padded(_bf(torch.randn(B, Cout, S, S, device=cuda_device)), 1, Cp)
    d_bits, d_mask = (ops.padded_empty(B, S, 1, Cp, cuda_device) for _ in range(2))
    ops.conv_fwd(dz, wd2, None, d_bits, 3, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mbits)
    ops.conv_fwd(dz, wd2, None, d_mask, 3, S, 1, 1, mode=ops.MODE_MASK, mask=yb)
    torch.cuda.synchronize()
    assert torch.equal(d_bits, d_mask)


def _fwd_fp8_160_case(ops, dev, B, seed=11, Cp=160):
    torch.manual_seed(seed)
    S, K = 19, 3
    C = 152 if Cp == 160 else Cp
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    xp = ops.to_padded(x, 1, Cp)
    ex = ops.fp8_exponent(float(x.abs().max()), margin=0)
    x8 = torch.empty(xp.shape, dtype=torch.uint8, device=dev)
    ops.quantize_fp8(xp, x8, ex)
    w8, ew = ops.pack_weights_fp8(torch.randn(C, C, K, K, device=dev) * 0.05, Cp, Cp)
    bp = F.pad(torch.randn(C, device=dev) * 0.1, (0, Cp - C))
    scales = torch.tensor([127 - ex, 127 - ew], dtype=torch.int32, device=dev)
    return x8, w8, bp, scales, torch.tensor([4.0], device=dev)


def _fwd_fp8_160_outputs(ops, dev, B, outs, Cp=160):
    S = 19
    y8 = torch.zeros((B, S + 2, S + 2, Cp), dtype=torch.uint8, device=dev)
    yb = ops.padded_empty(B, S, 1, Cp, dev) if outs == "both" else None
    mbits = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(Cp), dtype=torch.int32, device=dev)
    return y8, yb, mbits, ops.fp8_amax_buffer(1, dev)[0]


@pytest.mark.parametrize("Cp", [160, 192])
@pytest.mark.parametrize("B", [1, 37])
def test_conv_fwd_fp8_160_byte_outputs(ops, cuda_device, monkeypatch, B, Cp):
    """The fp8 training forward's e4m3-only output (staged through LDS, 16-B row stores, ragged
    last tile at B = 37) equals the e4m3 copy written next to a bf16 output, with the same ReLU'
    bitmask and amax, and leaves the zero border untouched."""
    monkeypatch.setenv("ALPHAGO_AMD_FP8_CW32", "1")
    S = 19
    x8, w8, bp, scales, osc = _fwd_fp8_160_case(ops, cuda_device, B, Cp=Cp)
    res = {}
    for outs in ("fp8", "both"):
        y8, yb, mbits, amax = _fwd_fp8_160_outputs(ops, cuda_device, B, outs, Cp=Cp)
        ops.conv_fwd_fp8(x8, w8, bp, scales, osc, 3, S, 1, 1, y_bf16=yb, y_fp8=y8, amax=amax, mbits=mbits)
        res[outs] = (y8, yb, mbits, amax)
    torch.cuda.synchronize()
    (y8a, _, mba, ama), (y8b, yb, mbb, amb) = res["fp8"], res["both"]
    assert torch.equal(y8a, y8b) and torch.equal(mba, mbb) and torch.equal(ama, amb)
    assert y8a[:, 0].sum() == 0 and y8a[:, :, 0].sum() == 0 and y8a[:, S + 1].sum() == 0
    assert y8a[:, :, S + 1].sum() == 0
    # the e4m3 bytes are the bf16 result's values at 4x (round-to-nearest of the fp32 value: within
    # one e4m3 step of the bf16-rounded copy)
    ref = ops.from_padded(yb, 1).float() * 4.0
    got = ops.fp8_to_float(y8a, 0)[:, 1:S + 1, 1:S + 1, :].permute(0, 3, 1, 2)
    assert ((got - ref).abs() <= ref.abs() * 0.07 + 1e-3).all()


@pytest.mark.parametrize("Cp,lab", [(160, 6), (192, 7)])
@pytest.mark.parametrize("B", lab_params([1, 5, 37], []))
def test_conv_fwd_fp8_160_matches_round4_tiling(ops, cuda_device, monkeypatch, B, Cp, lab):
    """Production fp8 forward with staged byte outputs (160: 4-wave workgroups too) == the
    round-4 tiling (lab 6 / 7: 8-wave workgroups, 4-B stores) byte for byte."""
    monkeypatch.setenv("ALPHAGO_AMD_FP8_CW32", "1")
    S = 19
    x8, w8, bp, scales, osc = _fwd_fp8_160_case(ops, cuda_device, B, Cp=Cp)
    y8, yb, mbits, amax = _fwd_fp8_160_outputs(ops, cuda_device, B, "both", Cp=Cp)
    ops.conv_fwd_fp8(x8, w8, bp, scales, osc, 3, S, 1, 1, y_bf16=yb, y_fp8=y8, amax=amax, mbits=mbits)
    y8l, ybl, mbl, aml = _fwd_fp8_160_outputs(ops, cuda_device, B, "both", Cp=Cp)
    ops.lab().conv_fwd_fp8(x8, w8, bp, scales, osc, aml, ybl, y8l, 3, S, 1, 1, lab, mbl)
    torch.cuda.synchronize()
    assert torch.equal(y8, y8l) and torch.equal(yb, ybl) and torch.equal(mbits, mbl)
    # amax slots follow the workgroup index (different grids): the maximum over the slots agrees
    assert amax.view(torch.float32).max().item() == aml.view(torch.float32).max().item()


@pytest.mark.parametrize("C,Cp", [(152, 160), (192, 192)])
@pytest.mark.parametrize("cw", [32, 64])
def test_conv_dgrad_fp8(ops, cuda_device, monkeypatch, cw, C, Cp):
    """fp8 dgrad (e5m2 gradients x transposed e4m3 weights on the block-scaled MFMA)
    masked by the bf16 activation vs fp32 conv2d_input of the dequantised operands."""
    monkeypatch.setenv("ALPHAGO_AMD_FP8_CW32", "1" if cw == 32 else "0")  # 160-channel packs: 32 / 64-channel chunks
    torch.manual_seed(4)
    B, S, K = 3, 19, 3
    dz = torch.randn(B, C, S, S, device=cuda_device) * 1e-3
    w = torch.randn(C, C, K, K, device=cuda_device) * 0.05
    yprev = _bf(torch.randn(B, C, S, S, device=cuda_device)).clamp_min(0)
    amax_in = ops.fp8_amax_buffer(1, cuda_device)[0]
    eg = ops.fp8_exponent(float(dz.abs().max()), margin=0) + 7  # e5m2 max 57344 = 448 * 2^7
    dzp = ops.to_padded(dz, 1, Cp)
    dz8 = torch.empty(dzp.shape, dtype=torch.uint8, device=cuda_device)
    ops.quantize_bf8(dzp, dz8, torch.tensor([2.0 ** eg], device=cuda_device), amax_in)
    assert abs(amax_in.view(torch.float32).max().item() - _bf(dz).abs().max().item()) < 1e-6
    ew = ops.fp8_exponent(float(w.abs().max()), margin=0)
    w8t = torch.zeros(ops.fp8_weight_shape(K, Cp, Cp), dtype=torch.uint8, device=cuda_device)
    ops.pack_weights_fp8_into(w, w8t, torch.tensor([2.0 ** ew], device=cuda_device), transposed=True)
    dzq = ops.bf8_to_float(dz8, eg)[:, 1:S + 1, 1:S + 1, :C].permute(0, 3, 1, 2)
    wq = (w * 2.0 ** ew).clamp(-448, 448).to(torch.float8_e4m3fn).float() * 2.0 ** -ew
    ref = torch.nn.grad.conv2d_input((B, C, S, S), wq, dzq, padding=K // 2) * (yprev > 0)
    scales = torch.tensor([127 - eg, 127 - ew], dtype=torch.int32, device=cuda_device)
    ey = ops.fp8_exponent(float(ref.abs().max()), margin=0) + 7
    osc = torch.tensor([2.0 ** ey], device=cuda_device)
    amax = ops.fp8_amax_buffer(1, cuda_device)[0]
    dx = ops.padded_empty(B, S, 1, Cp, cuda_device)
    dx8 = torch.zeros((B, S + 2, S + 2, Cp), dtype=torch.uint8, device=cuda_device)
    ops.conv_dgrad_fp8(dz8, w8t, ops.to_padded(yprev, 1, Cp), scales, osc, K, S, dx, y_fp8=dx8, amax=amax)
    torch.cuda.synchronize()
    out = ops.from_padded(dx, 1)
    assert _rel_err(out[:, :C], ref) < 1e-2
    assert out[:, C:].abs().sum() == 0
    assert _rel_err(ops.bf8_to_float(dx8, ey)[:, 1:S + 1, 1:S + 1, :C].permute(0, 3, 1, 2), ref) < 0.13
    assert abs(amax.view(torch.float32).max().item() - ref.abs().max().item()) <= 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("C,Cp,B", [(152, 160, 3), (192, 192, 3), (192, 192, 7)])
@pytest.mark.parametrize("cw", [32, 64])
def test_conv_dgrad_fp8_bf16_operand(ops, cuda_device, monkeypatch, cw, C, Cp, B):
    """fp8 dgrad straight from the bf16 gradient (converted to e5m2 in the kernel's registers,
    ReLU' from the forward's bitmask, bf16 output) vs fp32 conv2d_input of the dequantised
    operands: e5m2(dZ * 2^eg) * 2^-eg and e4m3 weights."""
    monkeypatch.setenv("ALPHAGO_AMD_FP8_CW32", "1" if cw == 32 else "0")  # 160-channel packs: 32 / 64-channel chunks
    torch.manual_seed(6)
    S, K = 19, 3
    xin = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w0 = _bf(torch.randn(C, C, K, K, device=cuda_device) * 0.05)
    b0 = torch.randn(C, device=cuda_device) * 0.1
    wp0 = ops.packed_weight_like(w0, Cp, Cp)
    ops.pack_weights([w0.contiguous()], [wp0])
    yprev = ops.padded_empty(B, S, 1, Cp, cuda_device)
    mbits = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(Cp), dtype=torch.int32, device=cuda_device)
    ops.conv_fwd(ops.to_padded(xin, 1, Cp), wp0, torch.nn.functional.pad(b0, (0, Cp - C)), yprev, K, S, 1, 1,
                 mbits=mbits)
    dz = _bf(torch.randn(B, C, S, S, device=cuda_device) * 1e-3)
    w = torch.randn(C, C, K, K, device=cuda_device) * 0.05
    eg = ops.fp8_exponent(float(dz.abs().max()), margin=0) + 7
    ew = ops.fp8_exponent(float(w.abs().max()), margin=0)
    w8t = torch.zeros(ops.fp8_weight_shape(K, Cp, Cp), dtype=torch.uint8, device=cuda_device)
    ops.pack_weights_fp8_multi([w], [w8t], torch.tensor([2.0 ** ew], device=cuda_device), [0], [1])
    dzq = (dz * 2.0 ** eg).clamp(-57344, 57344).to(torch.float8_e5m2).float() * 2.0 ** -eg
    wq = (w * 2.0 ** ew).clamp(-448, 448).to(torch.float8_e4m3fn).float() * 2.0 ** -ew
    ymask = ops.from_padded(yprev, 1)[:, :C] > 0
    ref = torch.nn.grad.conv2d_input((B, C, S, S), wq, dzq, padding=K // 2) * ymask
    scales = torch.tensor([127 - eg, 127 - ew], dtype=torch.int32, device=cuda_device)
    amax = ops.fp8_amax_buffer(1, cuda_device)[0]
    dx = ops.padded_empty(B, S, 1, Cp, cuda_device)
    ops.conv_dgrad_fp8_bf16(ops.to_padded(dz, 1, Cp), w8t, mbits, scales,
                            torch.tensor([2.0 ** eg], device=cuda_device), K, S, dx, amax=amax)
    torch.cuda.synchronize()
    out = ops.from_padded(dx, 1)
    assert _rel_err(out[:, :C], ref) < 1e-2
    assert out[:, C:].abs().sum() == 0
    assert dx[:, 0].abs().sum() == 0  # borders untouched
    assert abs(amax.view(torch.float32).max().item() - ref.abs().max().item()) <= 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("B,outs", [(3, "fp8"), (5, "bf16"), (2, "both")])
@pytest.mark.parametrize("cw", [32, 64])
def test_conv_dgrad_fp8_bits(ops, cuda_device, monkeypatch, cw, B, outs):
    """All-fp8 value backward: dgrad from the e5m2 dZ copy (the one the fp8 wgrad reads), ReLU' from
    the forward's bitmask, e5m2 and/or bf16 outputs vs fp32 conv2d_input of the dequantised operands."""
    monkeypatch.setenv("ALPHAGO_AMD_FP8_CW32", "1" if cw == 32 else "0")  # 160-channel packs: 32 / 64-channel chunks
    torch.manual_seed(16)
    S, K, C, Cp = 19, 3, 152, 160
    xin = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w0 = _bf(torch.randn(C, C, K, K, device=cuda_device) * 0.05)
    wp0 = ops.packed_weight_like(w0, Cp, Cp)
    ops.pack_weights([w0.contiguous()], [wp0])
    yprev = ops.padded_empty(B, S, 1, Cp, cuda_device)
    mbits = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(Cp), dtype=torch.int32, device=cuda_device)
    ops.conv_fwd(ops.to_padded(xin, 1, Cp), wp0, torch.randn(Cp, device=cuda_device) * 0.1, yprev, K, S, 1, 1,
                 mbits=mbits)
    dz = torch.randn(B, C, S, S, device=cuda_device) * 1e-3
    w = torch.randn(C, C, K, K, device=cuda_device) * 0.05
    eg = ops.fp8_exponent(float(dz.abs().max()), margin=0) + 7
    ew = ops.fp8_exponent(float(w.abs().max()), margin=0)
    w8t = torch.zeros(ops.fp8_weight_shape(K, Cp, Cp), dtype=torch.uint8, device=cuda_device)
    ops.pack_weights_fp8_multi([w], [w8t], torch.tensor([2.0 ** ew], device=cuda_device), [0], [1])
    dz8 = torch.zeros((B, S + 2, S + 2, Cp), dtype=torch.uint8, device=cuda_device)
    dz8[:, 1:S + 1, 1:S + 1, :C] = (dz * 2.0 ** eg).clamp(-57344, 57344).to(torch.float8_e5m2).view(
        torch.uint8).permute(0, 2, 3, 1)
    dzq = (dz * 2.0 ** eg).clamp(-57344, 57344).to(torch.float8_e5m2).float() * 2.0 ** -eg
    wq = (w * 2.0 ** ew).clamp(-448, 448).to(torch.float8_e4m3fn).float() * 2.0 ** -ew
    ymask = ops.from_padded(yprev, 1)[:, :C] > 0
    ref = torch.nn.grad.conv2d_input((B, C, S, S), wq, dzq, padding=K // 2) * ymask
    scales = torch.tensor([127 - eg, 127 - ew], dtype=torch.int32, device=cuda_device)
    eo = ops.fp8_exponent(float(ref.abs().max()), margin=0) + 7
    amax = ops.fp8_amax_buffer(1, cuda_device)[0]
    dx = ops.padded_empty(B, S, 1, Cp, cuda_device) if outs in ("bf16", "both") else None
    dx8 = torch.zeros_like(dz8) if outs in ("fp8", "both") else None
    ops.conv_dgrad_fp8_bits(dz8, w8t, mbits, scales, torch.tensor([2.0 ** eo], device=cuda_device), K, S,
                            y_bf16=dx, y_fp8=dx8, amax=amax)
    torch.cuda.synchronize()
    if dx is not None:
        out = ops.from_padded(dx, 1)
        assert _rel_err(out[:, :C], ref) < 1e-2
        assert out[:, C:].abs().sum() == 0
        assert dx[:, 0].abs().sum() == 0  # borders untouched
    if dx8 is not None:
        got = dx8[:, 1:S + 1, 1:S + 1, :C].view(torch.float8_e5m2).float().permute(0, 3, 1, 2) * 2.0 ** -eo
        # e5m2 keeps 2 mantissa bits: at most half a step (12.5 % of the value) from the fp32 result
        assert _rel_err(got, ref) < 0.13
        assert (got - ref).abs().mean().item() < 0.1 * ref.abs().mean().item()
        assert dx8[:, 0].sum() == 0 and dx8[:, 1:S + 1, 1:S + 1, C:].sum() == 0
    assert abs(amax.view(torch.float32).max().item() - ref.abs().max().item()) <= 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("Cin,Cout,K", [(152, 152, 3), (49, 152, 5), (192, 192, 3), (48, 192, 5)])
@pytest.mark.parametrize("cw", [32, 64])
def test_pack_weights_fp8_multi_matches_single(ops, cuda_device, monkeypatch, cw, Cin, Cout, K):
    """The one-launch fp8 repack equals the per-layer packs, forward and transposed."""
    monkeypatch.setenv("ALPHAGO_AMD_FP8_CW32", "1" if cw == 32 else "0")  # 160-channel packs: 32 / 64-channel chunks
    torch.manual_seed(8)
    w = torch.randn(Cout, Cin, K, K, device=cuda_device) * 0.05
    cout_p, cin_p = ops.pad_filters(Cout), (ops.pad_filters(Cin) if Cin > 64 else 64)
    sc = torch.tensor([4.0, 8.0], device=cuda_device)
    a = torch.zeros(ops.fp8_weight_shape(K, cin_p, cout_p), dtype=torch.uint8, device=cuda_device)
    b = torch.zeros_like(a)
    ops.pack_weights_fp8_into(w, a, sc[1:2])
    outs = [b]
    tr = Cin == Cout
    if tr:
        at = torch.zeros(ops.fp8_weight_shape(K, cout_p, cin_p), dtype=torch.uint8, device=cuda_device)
        bt = torch.zeros_like(at)
        ops.pack_weights_fp8_into(w, at, sc[1:2], transposed=True)
        outs.append(bt)
    ops.pack_weights_fp8_multi([w] * len(outs), outs, sc, [1] * len(outs), [0, 1][:len(outs)])
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    if tr:
        assert torch.equal(at, bt)


@pytest.mark.parametrize("B,S", [(3, 19), (7, 19), (24, 19), (5, 9)])
def test_conv_wgrad_fp8_160(ops, cuda_device, B, S):
    """fp8 wgrad (e5m2 dZ x e4m3 X, 128-pixel steps through ds_read_b64_tr_b8) vs fp32
    conv2d_weight of the dequantised operands; bias gradient from the e5m2 bytes (B = 24: the
    production 56 splits; S = 9: boards smaller than one 128-pixel step)."""
    torch.manual_seed(11)
    K, C, Cp = 3, 152, 160
    x = torch.relu(torch.randn(B, C, S, S, device=cuda_device)) * 2.0
    dz = torch.randn(B, C, S, S, device=cuda_device) * 1e-3
    ex = ops.fp8_exponent(float(x.abs().max()), margin=0)
    eg = ops.fp8_exponent(float(dz.abs().max()), margin=0) + 7
    xq = (x * 2.0 ** ex).clamp(-448, 448).to(torch.float8_e4m3fn).float() * 2.0 ** -ex
    dzq = (dz * 2.0 ** eg).clamp(-57344, 57344).to(torch.float8_e5m2).float() * 2.0 ** -eg
    x8 = torch.zeros((B, S + 2, S + 2, Cp), dtype=torch.uint8, device=cuda_device)
    x8[:, 1:S + 1, 1:S + 1, :C] = (x * 2.0 ** ex).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8).permute(0, 2, 3, 1)
    dz8 = torch.zeros_like(x8)
    dz8[:, 1:S + 1, 1:S + 1, :C] = (dz * 2.0 ** eg).clamp(-57344, 57344).to(torch.float8_e5m2).view(torch.uint8).permute(0, 2, 3, 1)
    ref_w = torch.nn.grad.conv2d_weight(xq, (C, C, K, K), dzq, padding=1)
    ref_b = dzq.sum(dim=(0, 2, 3))
    ns = ops.wgrad_fp8_nsplit(B * S * S)
    slab = torch.full((ns, K * K, Cp, Cp), float("nan"), device=cuda_device)
    dbs = torch.zeros(ns, Cp, device=cuda_device)
    xs = torch.tensor([127 - ex], dtype=torch.int32, device=cuda_device)
    gs = torch.tensor([127 - eg], dtype=torch.int32, device=cuda_device)
    gm = torch.tensor([2.0 ** eg], device=cuda_device)
    ops.conv_wgrad_fp8(x8, dz8, slab, dbs, xs, gs, gm, K, S, 1, 1)
    gw = torch.zeros(C, C, K, K, device=cuda_device)
    gb = torch.zeros(C, device=cuda_device)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert _rel_err(gw, ref_w) < 2e-3
    assert _rel_err(gb, ref_b) < 2e-3


def test_dgrad_bits_bf8_copy(ops, cuda_device):
    """The bitmask dgrad's e5m2 copy is e5m2(dx * scale) of the fp32 result (the bf16 output rounds
    the same value: rare one-step differences), and the amax slots hold max |dx|."""
    torch.manual_seed(12)
    B, S, K, C, Cp = 4, 19, 3, 152, 160
    xin = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w0 = _bf(torch.randn(C, C, K, K, device=cuda_device) * 0.05)
    wp0 = ops.packed_weight_like(w0, Cp, Cp)
    ops.pack_weights([w0], [wp0])
    y = ops.padded_empty(B, S, 1, Cp, cuda_device)
    mbits = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(Cp), dtype=torch.int32, device=cuda_device)
    ops.conv_fwd(ops.to_padded(xin, 1, Cp), wp0, torch.zeros(Cp, device=cuda_device), y, K, S, 1, 1, mbits=mbits)
    w = _bf(torch.randn(C, C, K, K, device=cuda_device) * 0.05)
    wf, wd = ops.packed_weight_like(w, Cp, Cp), ops.packed_weight_like(w, Cp, Cp, transposed=True)
    ops.pack_weights([w], [wf], [wd])
    dz = ops.to_padded(_bf(torch.randn(B, C, S, S, device=cuda_device) * 1e-3), 1, Cp)
    dx = ops.padded_empty(B, S, 1, Cp, cuda_device)
    dx8 = torch.zeros(dx.shape, dtype=torch.uint8, device=cuda_device)
    amax = ops.fp8_amax_buffer(1, cuda_device)[0]
    sc = torch.tensor([2.0 ** 20], device=cuda_device)
    ops.conv_dgrad_bits_bf8(dz, wd, dx, mbits, dx8, sc, K, S, amax=amax)
    ref = ops.padded_empty(B, S, 1, Cp, cuda_device)
    ops.conv_fwd(dz, wd, None, ref, K, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mbits)
    torch.cuda.synchronize()
    assert torch.equal(dx, ref)  # the bf16 output is unchanged by the extra copy
    q = (dx.float() * 2.0 ** 20).clamp(-57344, 57344).to(torch.float8_e5m2).view(torch.uint8)
    assert (q != dx8).float().mean().item() < 0.02  # fp32 vs bf16-rounded source: rare 1-ulp differences
    deq = dx8.view(torch.float8_e5m2).float() * 2.0 ** -20
    assert _rel_err(deq, dx.float()) < 0.13
    assert abs(amax.view(torch.float32).max().item() - dx.float().abs().max().item()) <= 1e-2 * dx.float().abs().max().item()


def test_fp8_weight_scales_matches_torch(ops, cuda_device):
    """Per-layer e4m3 weight exponents (16-B vector loads over the aligned prefix, scalar tail and
    misaligned views) == floor(log2(448 / max |w|)) from torch."""
    torch.manual_seed(21)
    flat = torch.randn(300000, device=cuda_device)
    ws = [flat[0:207936].view(152, 152, 3, 3), flat[1:186201],  # a misaligned view
          flat[200000:200000 + 1003] * 7.0, torch.randn(152, 49, 5, 5, device=cuda_device) * 1e-3]
    L = len(ws)
    wscale = torch.zeros(L, device=cuda_device)
    scales8 = torch.full((L, 2), 127, dtype=torch.int32, device=cuda_device)
    ops.fp8_weight_scales(ws, wscale, scales8)
    torch.cuda.synchronize()
    for l, w in enumerate(ws):
        m = w.abs().max().item()
        e = max(-60, min(60, math.floor(math.log2(448.0 / m))))
        assert wscale[l].item() == 2.0 ** e, (l, wscale[l].item(), e)
        assert scales8[l, 1].item() == 127 - e and scales8[l, 0].item() == 127
