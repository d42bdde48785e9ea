"""Numerics of the gfx950 HIP kernels vs plain PyTorch fp32 references."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _marks import LAB, lab_params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(cuda_device):
    from alphago_amd import ops as _ops

    _ops.load()
    return _ops


def _bf(x):
    return x.to(torch.bfloat16).float()


PROD_TILES = (0, 36, 37, 64, 128, 256, 384, 385, 386, 387)


def _conv_fwd(ops, tile, x, w, bias, y, K, S, Pin, Po=1, mode=0, mask=None, mbits=None):
    """Production tilings through torch.ops.alphago_amd, the kernel-lab ones
    through the separately built lab library (torch.ops.alphago_amd_lab)."""
    if tile in PROD_TILES:
        return ops.conv_fwd(x, w, bias, y, K, S, Pin, Po, mode=mode, mask=mask, mbits=mbits, tile=tile)
    ops.lab().conv_fwd(x, w, bias, mask, y, K, S, Pin, Po, mode, mbits, tile)
    return y


def _rel_err(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)


@pytest.mark.parametrize("B,Cin,Cout,K", [(5, 64, 192, 3), (3, 64, 192, 5), (4, 192, 192, 3), (7, 128, 128, 3), (2, 64, 64, 3)])
def test_conv_fwd_bias_relu(ops, cuda_device, B, Cin, Cout, K):
    torch.manual_seed(0)
    S, P = 19, K // 2
    x = _bf(torch.randn(B, Cin, S, S, device=cuda_device))
    w = _bf(torch.randn(Cout, Cin, K, K, device=cuda_device) * 0.05)
    b = torch.randn(Cout, device=cuda_device) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=P))
    xp = ops.to_padded(x, P)
    wp = ops.packed_weight_like(w, Cin, Cout)
    ops.pack_weights([w.contiguous()], [wp])
    y = ops.padded_empty(B, S, 1, Cout, cuda_device)
    ops.conv_fwd(xp, wp, b, y, K, S, P, 1)
    torch.cuda.synchronize()
    out = ops.from_padded(y, 1)
    assert _rel_err(out, ref) < 1e-2
    # borders untouched
    assert y[:, 0].abs().sum() == 0 and y[:, :, -1].abs().sum() == 0


def test_conv_fwd_asymmetric_identity(ops, cuda_device):
    """Tap/axis orientation check with an asymmetric single-tap kernel."""
    B, C, S = 1, 64, 19
    x = torch.zeros(B, C, S, S, device=cuda_device)
    x[0, 3, 5, 7] = 1.0
    w = torch.zeros(64, C, 3, 3, device=cuda_device)
    w[10, 3, 0, 2] = 2.0  # kh=0, kw=2
    ref = F.conv2d(x, w, padding=1)
    xp = ops.to_padded(x, 1)
    wp = ops.packed_weight_like(w, C, 64)
    ops.pack_weights([w], [wp])
    y = ops.padded_empty(B, S, 1, 64, cuda_device)
    ops.conv_fwd(xp, wp, torch.zeros(64, device=cuda_device), y, 3, S, 1, 1)
    out = ops.from_padded(y, 1)
    assert torch.equal(out, F.relu(ref))


@pytest.mark.parametrize("B,C,K", [(5, 192, 3), (3, 64, 3)])
def test_conv_dgrad_with_relu_mask(ops, cuda_device, B, C, K):
    torch.manual_seed(1)
    S = 19
    dz = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w = _bf(torch.randn(C, C, K, K, device=cuda_device) * 0.05)
    yprev = _bf(torch.randn(B, C, S, S, device=cuda_device)).clamp_min(0)  # post-ReLU activation
    # dx = conv_transpose(dz, w); masked by relu'(yprev)
    ref = torch.nn.grad.conv2d_input((B, C, S, S), w, dz, padding=K // 2) * (yprev > 0)
    wf = ops.packed_weight_like(w, C, C)
    wd = ops.packed_weight_like(w, C, C, transposed=True)
    ops.pack_weights([w], [wf], [wd])
    dzp = ops.to_padded(dz, 1)
    yp = ops.to_padded(yprev, 1)
    dx = ops.padded_empty(B, S, 1, C, cuda_device)
    ops.conv_fwd(dzp, wd, None, dx, K, S, 1, 1, mode=ops.MODE_MASK, mask=yp)
    out = ops.from_padded(dx, 1)
    assert _rel_err(out, ref) < 1e-2


@pytest.mark.parametrize("variant", lab_params([0, 14, 9, 5, 6, 7, 8, 1, 2, 3, 4], (0, 14)))
@pytest.mark.parametrize("B,Cin,Cout,K,Pin,nsplit", [(6, 192, 192, 3, 1, None), (5, 64, 192, 5, 2, None),
                                                    (3, 64, 64, 3, 1, None), (9, 128, 128, 3, 1, None),
                                                    (7, 192, 192, 3, 1, 1), (4, 192, 192, 3, 1, 3),
                                                    (11, 192, 192, 3, 1, 40), (2, 128, 128, 3, 1, 5)])
def test_conv_wgrad(ops, cuda_device, B, Cin, Cout, K, Pin, nsplit, variant):
    """variant 0: production per-tap kernel; 14: its small-batch plan (64 x 64 tap-merged tiles on any
    64-multiple 3x3 layer, ops.wgrad_config); 5: the one-kernel-row wgrad (conv_wgrad_row.hip) for
    192x192 and 128x128 3x3 layers; kernel-lab variants: 1-4, 6 tap-pair kernel for 192x192 3x3 (odd
    tap over split pairs; the slab starts as NaN, so every split's every tap must be written), 7
    per-tap kernel with whole-line staging, 8 tap pairs with the DMA spread through the MFMAs."""
    torch.manual_seed(2)
    S = 19
    x = _bf(torch.randn(B, Cin, S, S, device=cuda_device))
    dz = _bf(torch.randn(B, Cout, S, S, device=cuda_device))
    ref_w = torch.nn.grad.conv2d_weight(x, (Cout, Cin, K, K), dz, padding=K // 2)
    ref_b = dz.sum(dim=(0, 2, 3))
    xp = ops.to_padded(x, Pin)
    dzp = ops.to_padded(dz, 1)
    M = B * S * S
    ns = nsplit or ops.wgrad_splits(M, K * K)
    slab = torch.full((ns, K * K, Cout, Cin), float("nan"), device=cuda_device)
    dbs = torch.zeros(ns, Cout, device=cuda_device)
    if variant == 14 and (K != 3 or Pin != 1):
        pytest.skip("the small-batch plan covers 3x3 layers")
    if variant in (0, 14):  # production: per-tap kernel, 14 = its small-batch plan
        ops.conv_wgrad(xp, dzp, slab, dbs, K, S, Pin, 1, variant=variant)
    else:  # kernel-lab variants
        ops.lab().conv_wgrad(xp, dzp, slab, dbs, K, S, Pin, 1, 0, variant)
    gw = torch.zeros(Cout, Cin, K, K, device=cuda_device)
    gb = torch.zeros(Cout, device=cuda_device)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert _rel_err(gw, ref_w) < 2e-3
    assert _rel_err(gb, ref_b) < 2e-3


@pytest.mark.parametrize("S,B,Cin,Cin_real,Cout,K,Pin,ksub", [
    (19, 16, 192, 192, 192, 3, 1, 8), (19, 1, 192, 192, 192, 3, 1, 4), (19, 5, 192, 192, 192, 3, 1, 1),
    (19, 16, 64, 48, 192, 5, 2, 2), (13, 3, 64, 48, 128, 5, 2, 4), (9, 7, 128, 128, 128, 3, 1, 8),
    (19, 2, 64, 64, 64, 3, 1, 1), (19, 32, 192, 192, 192, 3, 1, 2), (9, 9, 160, 160, 160, 3, 1, 4)])
def test_conv_wgrad_direct(ops, cuda_device, S, B, Cin, Cin_real, Cout, K, Pin, ksub):
    """Split-free wgrad (kWgradDirect) straight into the OIHW gradient: fp32 reference, scale / beta
    accumulation, the first layer's 48 real planes of 64, other board sizes, and bitwise-equal repeats
    (one workgroup per output element, fixed pixel order)."""
    torch.manual_seed(11)
    assert ops.wgrad_direct_supported(Cout, Cin, Cin_real, K)
    x = _bf(torch.randn(B, Cin_real, S, S, device=cuda_device))
    dz = _bf(torch.randn(B, Cout, S, S, device=cuda_device))
    ref_w = torch.nn.grad.conv2d_weight(x, (Cout, Cin_real, K, K), dz, padding=K // 2)
    ref_b = dz.sum(dim=(0, 2, 3))
    xp = ops.to_padded(x, Pin, Cin)
    dzp = ops.to_padded(dz, 1)
    gw = torch.full((Cout, Cin_real, K, K), float("nan"), device=cuda_device)
    gb = torch.full((Cout,), float("nan"), device=cuda_device)
    ops.conv_wgrad_direct(xp, dzp, gw, gb, K, S, Pin, 1, ksub=ksub)  # beta 0: NaN never read
    torch.cuda.synchronize()
    assert _rel_err(gw, ref_w) < 2e-3
    assert _rel_err(gb, ref_b) < 2e-3
    gw2 = gw.clone()
    gb2 = gb.clone()
    ops.conv_wgrad_direct(xp, dzp, gw2, gb2, K, S, Pin, 1, scale=0.5, beta=2.0, ksub=ksub)
    torch.cuda.synchronize()
    assert _rel_err(gw2, 2.5 * gw) < 1e-5 and _rel_err(gb2, 2.5 * gb) < 1e-5
    gw3 = torch.zeros_like(gw)
    gb3 = torch.zeros_like(gb)
    ops.conv_wgrad_direct(xp, dzp, gw3, gb3, K, S, Pin, 1, ksub=ksub)
    torch.cuda.synchronize()
    assert torch.equal(gw3, gw) and torch.equal(gb3, gb)


@pytest.mark.parametrize("S,B,Cin,Cin_real,Cout,K,Pin", [(9, 13, 192, 192, 192, 3, 1), (13, 6, 192, 192, 192, 3, 1),
                                                         (9, 7, 64, 48, 192, 5, 2), (13, 3, 64, 48, 128, 5, 2),
                                                         (19, 1, 128, 128, 128, 3, 1)])
@LAB
def test_conv_wgrad_row_kernel_boards(ops, cuda_device, S, B, Cin, Cin_real, Cout, K, Pin):
    """The one-kernel-row wgrad at other board sizes (windows of 32 compact pixels cross board rows
    and boards at every alignment; taps leaving the board read the LDS zero rows), with the split
    count of the training engine."""
    torch.manual_seed(7)
    L = ops.lab()
    assert L.wgrad_plan(Cout, Cin, Cin_real, K, 5)[0] == K  # the row kernel applies
    x = _bf(torch.randn(B, Cin_real, S, S, device=cuda_device))
    dz = _bf(torch.randn(B, Cout, S, S, device=cuda_device))
    ref_w = torch.nn.grad.conv2d_weight(x, (Cout, Cin_real, K, K), dz, padding=K // 2)
    ref_b = dz.sum(dim=(0, 2, 3))
    xp = ops.to_padded(x, Pin, Cin)
    dzp = ops.to_padded(dz, 1)
    ns = ops.wgrad_splits(B * S * S, K * K // K)
    slab = torch.full((ns, K * K, Cout, Cin), float("nan"), device=cuda_device)
    dbs = torch.zeros(ns, Cout, device=cuda_device)
    L.conv_wgrad(xp, dzp, slab, dbs, K, S, Pin, 1, Cin_real if Cin_real < Cin else 0, 5)
    gw = torch.zeros(Cout, Cin_real, K, K, device=cuda_device)
    gb = torch.zeros(Cout, device=cuda_device)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert _rel_err(gw, ref_w) < 2e-3
    assert _rel_err(gb, ref_b) < 2e-3


@pytest.mark.parametrize("variant", [6, 7, 8])
@pytest.mark.parametrize("S,B", [(9, 13), (13, 6), (19, 2176)])
@LAB
def test_conv_wgrad_line_lab_boards(ops, cuda_device, S, B, variant):
    """The kernel-lab line-staged wgrads (6 / 8: tap pairs, 4.5 workgroups per split, one per CU;
    7: per tap) at other board sizes and at the SL bench batch, with a one-round split count."""
    torch.manual_seed(8)
    C = 192
    x = _bf(torch.randn(B, C, S, S, device=cuda_device))
    dz = _bf(torch.randn(B, C, S, S, device=cuda_device))
    ref_w = torch.nn.grad.conv2d_weight(x.float(), (C, C, 3, 3), dz.float(), padding=1)
    ref_b = dz.float().sum(dim=(0, 2, 3))
    xp = ops.to_padded(x, 1)
    dzp = ops.to_padded(dz, 1)
    L = ops.lab()
    t_, per_split, per_cu = (int(v) for v in L.wgrad_plan(C, C, 0, 3, variant)[:3])
    ns = max(1, min(256 * per_cu // per_split, (B * S * S + 31) // 32 // ops.WGRAD_MIN_STAGES))
    slab = torch.full((ns, 9, C, C), float("nan"), device=cuda_device)
    dbs = torch.zeros(ns, C, device=cuda_device)
    L.conv_wgrad(xp, dzp, slab, dbs, 3, S, 1, 1, 0, variant)
    gw = torch.zeros(C, C, 3, 3, device=cuda_device)
    gb = torch.zeros(C, device=cuda_device)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert _rel_err(gw, ref_w) < 2e-3
    assert _rel_err(gb, ref_b) < 2e-3


@pytest.mark.parametrize("K,Pin,variant,S,B,Cout", [(5, 2, 0, 19, 5, 192), (3, 1, 0, 19, 5, 192)] +
                         [(5, 2, v, S, B, C) for v in (10, 11, 12)
                          for S, B, C in ((19, 5, 192), (9, 13, 192), (13, 3, 128), (19, 1, 64))])
def test_conv_wgrad_thin_input(ops, cuda_device, K, Pin, variant, S, B, Cout):
    """48 real input planes padded to 64 (the policy net's first layer): the
    cin_real path computes only the real channels, matching the fp32 reference (variants 10-12: the
    kernel rows on 12 waves (4 n x 3 c) / with unit pipelining / both)."""
    torch.manual_seed(5)
    Cin = 48
    x = _bf(torch.randn(B, Cin, S, S, device=cuda_device))
    dz = _bf(torch.randn(B, Cout, S, S, device=cuda_device))
    ref_w = torch.nn.grad.conv2d_weight(x, (Cout, Cin, K, K), dz, padding=K // 2)
    ref_b = dz.sum(dim=(0, 2, 3))
    xp = ops.to_padded(x, Pin, 64)
    dzp = ops.to_padded(dz, 1)
    ns = ops.wgrad_splits(B * S * S, K * K)
    slab = torch.full((ns, K * K, Cout, 64), float("nan"), device=cuda_device)  # unwritten columns must be ignored
    dbs = torch.zeros(ns, Cout, device=cuda_device)
    ops.conv_wgrad(xp, dzp, slab, dbs, K, S, Pin, 1, cin_real=Cin, variant=variant)
    gw = torch.zeros(Cout, Cin, K, K, device=cuda_device)
    gb = torch.zeros(Cout, device=cuda_device)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert _rel_err(gw, ref_w) < 2e-3
    assert _rel_err(gb, ref_b) < 2e-3


# B = 7: 1024-thread BoardRegs; B = 300: 512-thread BoardRows (S * C / 8 <= 512) or, at C = 256,
# the 1024-thread fallback; S = 9 covers boards smaller than the register tiles
@pytest.mark.parametrize("C,B,S", [(192, 7, 19), (64, 7, 19), (128, 7, 19), (192, 300, 19), (256, 300, 19),
                                   (64, 300, 9), (192, 7, 9)])
def test_policy_head_train(ops, cuda_device, C, B, S):
    torch.manual_seed(3)
    y = _bf(torch.randn(B, C, S, S, device=cuda_device)).clamp_min(0)
    w = torch.randn(C, device=cuda_device) * 0.05
    b = torch.randn(1, device=cuda_device)
    tgt = torch.randint(0, S * S, (B,), device=cuda_device, dtype=torch.int32)
    tgt[2] = -1  # no target
    yr = y.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    logits = (yr * wr.view(1, C, 1, 1)).sum(1).flatten(1) + br
    valid = tgt >= 0
    lossv = F.cross_entropy(logits[valid], tgt[valid].long(), reduction="none")
    (lossv.sum() / B).backward()
    yp = ops.to_padded(y, 1)
    dz = ops.padded_empty(B, S, 1, C, cuda_device)
    loss = torch.empty(B, device=cuda_device)
    corr = torch.empty(B, device=cuda_device)
    dh = torch.empty(B, C + 1, device=cuda_device)
    ops.policy_head_train(yp, w, b, tgt, dz, loss, corr, dh, S, 1.0 / B)
    torch.cuda.synchronize()
    assert torch.allclose(loss[valid], lossv.detach(), rtol=1e-3, atol=1e-4)
    assert loss[2].item() == 0
    acc_ref = (logits.argmax(1) == tgt.long()).float() * valid
    assert torch.equal(corr, acc_ref)
    dzr = yr.grad * (y > 0)
    assert _rel_err(ops.from_padded(dz, 1), dzr) < 1e-2
    assert _rel_err(dh[:, :C].sum(0), wr.grad) < 1e-3
    assert abs(dh[:, C].sum().item() - br.grad.item()) < 1e-4


def test_policy_head_probs_legal(ops, cuda_device):
    torch.manual_seed(4)
    B, C, S = 3, 128, 19
    y = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w = torch.randn(C, device=cuda_device) * 0.1
    b = torch.zeros(1, device=cuda_device)
    legal = (torch.rand(B, S * S, device=cuda_device) > 0.3).to(torch.uint8)
    logits = (y * w.view(1, C, 1, 1)).sum(1).flatten(1)
    ref = torch.softmax(logits.masked_fill(legal == 0, float("-inf")), 1)
    probs = torch.empty(B, S * S, device=cuda_device)
    ops.policy_head_probs(ops.to_padded(y, 1), w, b, probs, S, legal=legal)
    assert torch.allclose(probs, ref, atol=1e-5)


# (48, 19, 64): per-board LDS kernel, 4-byte loads; (3, 9, 8): its byte loads (243 bytes per board);
# (200, 19, 208): 72 KB per board, the grid-stride kernel
@pytest.mark.parametrize("C,S,Cp", [(48, 19, 64), (3, 9, 8), (200, 19, 208)])
def test_pack_input_symmetries(ops, cuda_device, C, S, Cp):
    torch.manual_seed(5)
    B = 8
    planes = torch.randint(0, 256, (B, C, S, S), dtype=torch.uint8)
    sym = torch.arange(8, dtype=torch.int32)
    tgt = torch.randint(0, S * S, (B,), dtype=torch.int32)
    tf = [lambda a: a, lambda a: np.rot90(a, 1), lambda a: np.rot90(a, 2), lambda a: np.rot90(a, 3),
          lambda a: np.fliplr(a), lambda a: np.flipud(a), lambda a: np.transpose(a), lambda a: np.fliplr(np.rot90(a, 1))]
    out = ops.padded_empty(B, S, 2, Cp, cuda_device)
    tout = torch.empty(B, dtype=torch.int32, device=cuda_device)
    ops.pack_input(planes.to(cuda_device), out, 2, sym=sym.to(cuda_device), target=tgt.to(cuda_device), target_out=tout)
    assert not ops.from_padded(out, 2)[:, C:].any()  # channels past the real planes are zero
    got = ops.from_padded(out, 2, C).float().cpu().numpy()
    for b in range(B):
        exp = np.stack([tf[b](planes[b, c].numpy()) for c in range(C)])
        assert np.array_equal(got[b], exp), "symmetry %d" % b
        onehot = np.zeros((S, S))
        onehot[divmod(int(tgt[b]), S)] = 1
        assert int(np.argmax(tf[b](onehot))) == int(tout[b])


@pytest.mark.parametrize("C,Cp", [(48, 64), (49, 64), (200, 208)])
def test_pack_input_rows_gather(ops, cuda_device, C, Cp):
    """rows: the pack kernel gathers pool[rows] itself -- equal to index_select then pack, and a row
    outside the pool packs an all-zero board instead of reading out of bounds."""
    torch.manual_seed(6)
    S, npool, B = 19, 50, 9
    pool = torch.randint(0, 256, (npool, C, S, S), dtype=torch.uint8, device=cuda_device)
    rows = torch.randint(0, npool, (B,), device=cuda_device)
    sym = torch.randint(0, 8, (B,), dtype=torch.int32, device=cuda_device)
    tgt = torch.randint(0, S * S, (B,), dtype=torch.int32, device=cuda_device)
    ref, got = (ops.padded_empty(B, S, 2, Cp, cuda_device) for _ in range(2))
    tref, tgot = (torch.empty(B, dtype=torch.int32, device=cuda_device) for _ in range(2))
    ops.pack_input(pool.index_select(0, rows), ref, 2, sym=sym, target=tgt, target_out=tref)
    ops.pack_input(pool, got, 2, sym=sym, target=tgt, target_out=tgot, rows=rows)
    assert torch.equal(got, ref) and torch.equal(tgot, tref)
    bad = rows.clone()
    bad[3], bad[5] = npool, -1
    ops.pack_input(pool, got, 2, sym=sym, rows=bad)
    torch.cuda.synchronize()
    assert not got[3].any() and not got[5].any()
    keep = [b for b in range(B) if b not in (3, 5)]
    assert torch.equal(got[keep], ref[keep])


@pytest.mark.parametrize("C", [48, 49])
def test_pack_input_e4m3_copy(ops, cuda_device, C):
    """out8: the pack writes the e4m3 copy the fp8 trunk reads -- quantize_fp8(out, ., 0)'s bytes
    (plane values 0-255: exact up to 16, saturating at 448), borders untouched."""
    torch.manual_seed(7)
    S, B = 19, 5
    planes = torch.randint(0, 256, (B, C, S, S), dtype=torch.uint8, device=cuda_device)
    planes[:2] = planes[:2] & 1  # binary boards as in training
    sym = torch.randint(0, 8, (B,), dtype=torch.int32, device=cuda_device)
    out = ops.padded_empty(B, S, 2, 64, cuda_device)
    got8 = torch.zeros(out.shape, dtype=torch.uint8, device=cuda_device)
    ops.pack_input(planes, out, 2, sym=sym, out8=got8)
    ref8 = torch.zeros_like(got8)
    ops.quantize_fp8(out, ref8, 0)
    torch.cuda.synchronize()
    assert torch.equal(got8, ref8)
    assert torch.equal(got8[:2].view(torch.float8_e4m3fn).float(), out[:2].float())  # 0/1 planes: exact


def test_sgd_update(ops, cuda_device):
    p = torch.randn(1003, device=cuda_device)
    g = torch.randn(1003, device=cuda_device)
    ref = p - 0.01 * 0.5 * g
    ops.sgd_update(p, g, 0.01, 0.5)
    assert torch.allclose(p, ref)


@pytest.mark.parametrize("tile", lab_params([36, 37, 64, 65, 128, 130, 256, 2568, -1, 32, 2, 384, 385, 386, 387, 4, 5, 6, 7,
                                             8, 9, 10, 11], PROD_TILES))
def test_conv_fwd_tile_variants(ops, cuda_device, tile):
    """Every forward tiling (gather 128/256, 128-pixel waves, halo) on a batch
    whose pixel count is not a multiple of any tile."""
    torch.manual_seed(1)
    B, C, S = 9, 192, 19
    x = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w = _bf(torch.randn(C, C, 3, 3, device=cuda_device) * 0.05)
    b = torch.randn(C, device=cuda_device) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    xp = ops.to_padded(x, 1)
    wp = ops.packed_weight_like(w, C, C)
    ops.pack_weights([w.contiguous()], [wp])
    y = ops.padded_empty(B, S, 1, C, cuda_device)
    _conv_fwd(ops, tile, xp, wp, b, y, 3, S, 1, 1)
    torch.cuda.synchronize()
    assert _rel_err(ops.from_padded(y, 1), ref) < 1e-2
    assert y[:, 0].abs().sum() == 0 and y[:, :, -1].abs().sum() == 0


@pytest.mark.parametrize("tile", lab_params([36, 37, 64, 65, 130, 32, 256, 2, 384, 385, 386, 387, 4, 5, 6, 7, 8, 9, 10, 11],
                                            PROD_TILES))
def test_conv_ring_5x5_and_dgrad(ops, cuda_device, tile):
    """Layer-1 geometry (Cin 64, 5x5, input pad 2) and the masked dgrad mode on each tiling."""
    torch.manual_seed(2)
    B, S = 7, 19
    x = _bf(torch.randn(B, 64, S, S, device=cuda_device))
    w = _bf(torch.randn(192, 64, 5, 5, device=cuda_device) * 0.05)
    b = torch.randn(192, device=cuda_device) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=2))
    xp = ops.to_padded(x, 2)
    wp = ops.packed_weight_like(w, 64, 192)
    ops.pack_weights([w.contiguous()], [wp])
    y = ops.padded_empty(B, S, 1, 192, cuda_device)
    g = _bf(torch.randn(B, 192, S, S, device=cuda_device))
    w3 = _bf(torch.randn(192, 192, 3, 3, device=cuda_device) * 0.05)
    mask = _bf(torch.randn(B, 192, S, S, device=cuda_device)).relu()
    wd = ops.packed_weight_like(w3, 192, 192, True)
    wf = ops.packed_weight_like(w3, 192, 192)
    ops.pack_weights([w3.contiguous()], [wf], [wd])
    dx = ops.padded_empty(B, S, 1, 192, cuda_device)
    _conv_fwd(ops, tile, xp, wp, b, y, 5, S, 2, 1)
    _conv_fwd(ops, tile, ops.to_padded(g, 1), wd, None, dx, 3, S, 1, 1, mode=ops.MODE_MASK, mask=ops.to_padded(mask, 1))
    torch.cuda.synchronize()
    assert _rel_err(ops.from_padded(y, 1), ref) < 1e-2
    ref_dx = torch.nn.grad.conv2d_input(x.shape[:1] + (192, S, S), w3, g, padding=1) * (mask > 0)
    assert _rel_err(ops.from_padded(dx, 1), ref_dx) < 1e-2


@pytest.mark.parametrize("variant", lab_params([0, 1, 3, 4, 5], (0,)))
@pytest.mark.parametrize("K,Cin,Cout,B", [(3, 192, 192, 5), (5, 64, 192, 3), (3, 128, 128, 4), (3, 192, 64, 2)])
def test_conv_fwd_fp8(ops, cuda_device, K, Cin, Cout, B, variant):
    """e4m3 conv on the block-scaled MFMA vs fp32 conv of the dequantised operands
    (variant 0: production, pixel operand loaded from L2 into registers; lab:
    1/3/4 other tilings of it, 5 LDS-staged operands)."""
    _check_conv_fwd_fp8(ops, cuda_device, K, Cin, Cout, B, variant)


def _check_conv_fwd_fp8(ops, cuda_device, K, Cin, Cout, B, variant=0):
    torch.manual_seed(3)
    S, P = 19, K // 2
    x = F.relu(torch.randn(B, Cin, S, S, device=cuda_device)) * 3.0
    w = torch.randn(Cout, Cin, K, K, device=cuda_device) * 0.05
    b = torch.randn(Cout, device=cuda_device) * 0.1
    xp = ops.to_padded(x, P)
    ex = ops.fp8_exponent(float(x.abs().max()), margin=0)
    x8 = torch.empty(xp.shape, dtype=torch.uint8, device=cuda_device)
    ops.quantize_fp8(xp, x8, ex)
    w8, ew = ops.pack_weights_fp8(w, Cout, Cin)
    # dequantised operands (what the MFMA multiplies)
    xq = ops.fp8_to_float(x8, ex)[:, P:P + S, P:P + S, :Cin].permute(0, 3, 1, 2)
    wq = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, 0)).mul(2.0 ** ew).clamp(-448, 448)
    wq = wq.to(torch.float8_e4m3fn).float() * 2.0 ** -ew
    ref = F.relu(F.conv2d(xq, wq, b, padding=P))
    scales = torch.tensor([127 - ex, 127 - ew], dtype=torch.int32, device=cuda_device)
    ey = ops.fp8_exponent(float(ref.max()), margin=0)
    osc = torch.tensor([2.0 ** ey], device=cuda_device)
    amax = ops.fp8_amax_buffer(1, cuda_device)[0]
    yb = ops.padded_empty(B, S, 1, Cout, cuda_device)
    y8 = torch.zeros((B, S + 2, S + 2, Cout), dtype=torch.uint8, device=cuda_device)
    if variant == 0:
        ops.conv_fwd_fp8(x8, w8, b, scales, osc, K, S, P, 1, y_bf16=yb, y_fp8=y8, amax=amax)
    else:
        ops.lab().conv_fwd_fp8(x8, w8, b, scales, osc, amax, yb, y8, K, S, P, 1, variant)
    torch.cuda.synchronize()
    assert _rel_err(ops.from_padded(yb, 1), ref) < 1e-2
    assert _rel_err(ops.fp8_to_float(y8, ey)[:, 1:S + 1, 1:S + 1].permute(0, 3, 1, 2), ref) < 0.07
    assert abs(amax.view(torch.float32).max().item() - ref.max().item()) <= 1e-2 * ref.max().item()
    assert y8[:, 0].sum() == 0 and yb[:, :, -1].abs().sum() == 0


@pytest.mark.parametrize("tile", lab_params([0, 36, 37, 64, 65, 128, 130, 256, 384, 385, 386, 387, 32, 2, 4, 5, 6, 7, 8, 9,
                                             10, 11], PROD_TILES))
@pytest.mark.parametrize("C", [192, 128])
def test_relu_bitmask_dgrad_matches_mask(ops, cuda_device, tile, C):
    """Forward writes the ReLU' bitmask; dgrad mode 3 (bitmask) == mode 1 (bf16 activation mask)."""
    torch.manual_seed(4)
    B, S = 6, 19
    x = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w = _bf(torch.randn(C, C, 3, 3, device=cuda_device) * 0.05)
    b = torch.randn(C, device=cuda_device) * 0.1
    wf = ops.packed_weight_like(w, C, C)
    wd = ops.packed_weight_like(w, C, C, True)
    ops.pack_weights([w.contiguous()], [wf], [wd])
    xp = ops.to_padded(x, 1)
    y = ops.padded_empty(B, S, 1, C, cuda_device)
    mb = torch.full((B * (S + 2) ** 2 * ops.mbits_words(C),), -1, dtype=torch.int32, device=cuda_device)
    g = ops.to_padded(_bf(torch.randn(B, C, S, S, device=cuda_device)), 1)
    d1 = ops.padded_empty(B, S, 1, C, cuda_device)
    d3 = ops.padded_empty(B, S, 1, C, cuda_device)
    _conv_fwd(ops, tile, xp, wf, b, y, 3, S, 1, 1, mbits=mb)
    _conv_fwd(ops, tile, g, wd, None, d1, 3, S, 1, 1, mode=ops.MODE_MASK, mask=y)
    _conv_fwd(ops, tile, g, wd, None, d3, 3, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mb)
    torch.cuda.synchronize()
    assert _rel_err(ops.from_padded(y, 1), F.relu(F.conv2d(x, w, b, padding=1))) < 1e-2
    assert torch.equal(d1, d3)
    assert (ops.from_padded(d3, 1) != 0).any()


@pytest.mark.parametrize("ns,T,Cout,Cin,Cin_real,Cout_real", [(1, 9, 192, 192, 192, 192), (3, 9, 64, 64, 64, 64),
                                                            (7, 25, 192, 64, 48, 192), (56, 9, 192, 192, 192, 192),
                                                            (21, 9, 192, 192, 192, 152), (5, 25, 192, 64, 49, 192)])
def test_conv_wgrad_reduce_vs_fp32(ops, cuda_device, ns, T, Cout, Cin, Cin_real, Cout_real):
    """Split-K reduce alone: any split count (incl. < 4 and not a multiple of 4),
    thin input (NaN in the unused slab columns), padded Cout, scale and beta
    (accumulate into an existing gradient), bit-identical when repeated."""
    torch.manual_seed(11)
    K = int(round(T ** 0.5))
    slab = torch.randn(ns, T, Cout, Cin, device=cuda_device)
    slab[..., Cin_real:] = float("nan")
    dbs = torch.randn(ns, Cout, device=cuda_device)
    ref_w = slab[:, :, :Cout_real, :Cin_real].double().sum(0).permute(1, 2, 0).reshape(Cout_real, Cin_real, K, K)
    ref_b = dbs[:, :Cout_real].double().sum(0)
    g0w = torch.randn(Cout_real, Cin_real, K, K, device=cuda_device)
    g0b = torch.randn(Cout_real, device=cuda_device)
    outs = []
    for _ in range(2):
        gw, gb = g0w.clone(), g0b.clone()
        ops.conv_wgrad_reduce(slab, dbs, gw, gb, 0.5, 2.0)
        outs.append((gw, gb))
    torch.cuda.synchronize()
    exp_w = 2.0 * g0w.double() + 0.5 * ref_w
    exp_b = 2.0 * g0b.double() + 0.5 * ref_b
    assert (outs[0][0].double() - exp_w).abs().max().item() < 1e-4 * max(1.0, ns ** 0.5)
    assert (outs[0][1].double() - exp_b).abs().max().item() < 1e-4 * max(1.0, ns ** 0.5)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    gw = torch.full_like(g0w, float("nan"))  # beta 0 overwrites (never reads) the destination
    gb = torch.zeros_like(g0b)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert torch.isfinite(gw).all()
    assert (gw.double() - ref_w).abs().max().item() < 1e-4 * max(1.0, ns ** 0.5)


def test_bad_launch_raises(ops, cuda_device):
    """A launch the runtime rejects surfaces as a Python RuntimeError (every op
    runs launch_check after its kernels), not as silently unwritten output."""
    with pytest.raises(RuntimeError, match="launch failed"):
        torch.ops.alphago_amd.selftest_bad_launch()
    # the error is consumed: the next op runs normally
    p, g = torch.ones(8, device=cuda_device), torch.ones(8, device=cuda_device)
    ops.sgd_update(p, g, 0.5, 1.0)
    assert torch.allclose(p, torch.full_like(p, 0.5))


def test_production_library_has_no_lab_variants(ops, cuda_device):
    """Kernel-lab tilings/variants are not compiled into the production library:
    asking for one raises instead of switching kernels."""
    assert not torch.ops.alphago_amd.is_debug_build()
    x = ops.padded_empty(1, 19, 1, 64, cuda_device)
    w = torch.zeros(9, 64, 64, dtype=torch.bfloat16, device=cuda_device)
    y = ops.padded_empty(1, 19, 1, 64, cuda_device)
    for tile in (11, 65, 130):  # 65 / 130: the LDS-ring tiles, retired in round 5
        with pytest.raises(RuntimeError, match="not a production tiling"):
            ops.conv_fwd(x, w, torch.zeros(64, device=cuda_device), y, 3, 19, 1, 1, tile=tile)
    assert not hasattr(torch.ops.alphago_amd, "set_conv_tile")
    # round 5: the packed-tap first layer, the ring wgrad (9) and the first-layer wgrad re-cuts (10-13)
    # are lab-only; the production op refuses the variants, and the library has no conv_fwd_pk op
    assert not hasattr(torch.ops.alphago_amd, "conv_fwd_pk")
    x64 = ops.padded_empty(2, 19, 2, 64, cuda_device)
    dz = ops.padded_empty(2, 19, 1, 192, cuda_device)
    slab = torch.zeros(1, 25, 192, 64, device=cuda_device)
    dbs = torch.zeros(1, 192, device=cuda_device)
    for variant in (9, 10, 11, 12, 13):
        with pytest.raises((RuntimeError, ValueError), match="kernel-lab"):
            torch.ops.alphago_amd.conv_wgrad(x64, dz, slab, dbs, 5, 19, 2, 1, 48, variant)
    import subprocess

    from alphago_amd import _build

    # the retired packed-tap launcher is not in the production library
    syms = subprocess.run(["nm", "-D", "-C", _build.hip_path("prod")], capture_output=True, text=True).stdout
    assert "launch_conv_fwd_pk" not in syms


_DEBUG_CHILD = r"""
import torch, torch.nn.functional as F
from alphago_amd import ops
ops.load(build_if_missing=False)
assert torch.ops.alphago_amd.is_debug_build()
dev = torch.device("cuda:0")
torch.manual_seed(0)
B, C, S = 5, 192, 19
x = torch.randn(B, C, S, S, device=dev).bfloat16().float()
w = (torch.randn(C, C, 3, 3, device=dev) * 0.05).bfloat16().float()
b = torch.randn(C, device=dev) * 0.1
xp = ops.to_padded(x, 1)
wf = ops.packed_weight_like(w, C, C); wd = ops.packed_weight_like(w, C, C, True)
ops.pack_weights([w.contiguous()], [wf], [wd])
y = ops.padded_empty(B, S, 1, C, dev)
mb = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(C), dtype=torch.int32, device=dev)
ops.conv_fwd(xp, wf, b, y, 3, S, 1, 1, mbits=mb)          # bounds-checked forward
ref = F.relu(F.conv2d(x, w, b, padding=1))
err = (ops.from_padded(y, 1) - ref).abs().max().item() / ref.abs().max().item()
assert err < 1e-2, err
d = ops.padded_empty(B, S, 1, C, dev)
ops.conv_fwd(y, wd, None, d, 3, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mb)  # bounds-checked dgrad
ns = ops.wgrad_splits(B * S * S, 9)
slab = torch.empty(ns, 9, C, C, device=dev); dbs = torch.zeros(ns, C, device=dev)
ops.conv_wgrad(xp, y, slab, dbs, 3, S, 1, 1)               # bounds-checked wgrad
try:
    torch.ops.alphago_amd.debug_conv_fwd_understated(xp, wf, b, y, 3, S, 1, 1)
except RuntimeError as e:
    assert "bounds check failed" in str(e), e
    print("DEBUG-OK")
else:
    raise SystemExit("device bounds check did not fire")
"""


def test_debug_build_bounds_checks(cuda_device, tmp_path):
    """The AGK_DEBUG library (device bounds checks in the conv kernels) runs the
    forward, bitmask dgrad and wgrad of a real layer clean, and an understated
    tensor extent makes the next op raise a RuntimeError naming the check."""
    import os
    import subprocess
    import sys
    from alphago_amd import _build
    if not os.path.exists(_build.hip_path("debug")):
        pytest.skip("debug library not built")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ALPHAGO_AMD_KERNELS="debug", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", _DEBUG_CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "DEBUG-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("M,N,K,ta,tb,bias,beta", [(2176, 256, 361, False, False, True, 0.0),
                                                   (361, 256, 2176, True, False, False, 0.0),
                                                   (2176, 361, 256, False, True, False, 0.0),
                                                   (37, 70, 5, False, False, True, 0.5),
                                                   (81, 16, 9, True, True, False, 1.0)])
def test_dense_f32_vs_torch(ops, cuda_device, M, N, K, ta, tb, bias, beta):
    """Value-head dense GEMM (fp32 MFMA) vs fp64 torch: the three shapes of the
    value head (forward, dW1 = z^T dh, dz = dh W1^T) and ragged/transposed ones."""
    torch.manual_seed(9)
    A = torch.randn((K, M) if ta else (M, K), device=cuda_device)
    B = torch.randn((N, K) if tb else (K, N), device=cuda_device)
    b = torch.randn(N, device=cuda_device) if bias else None
    C0 = torch.randn(M, N, device=cuda_device)
    C = C0.clone()
    ops.dense_f32(A, B, C, bias=b, trans_a=ta, trans_b=tb, beta=beta)
    ref = (A.double().t() if ta else A.double()) @ (B.double().t() if tb else B.double())
    if bias:
        ref = ref + b.double()
    ref = ref + beta * C0.double()
    torch.cuda.synchronize()
    assert (C.double() - ref).abs().max().item() < 1e-5 * max(1.0, K ** 0.5) * ref.abs().max().item()
    C2 = C0.clone()
    ops.dense_f32(A, B, C2, bias=b, trans_a=ta, trans_b=tb, beta=beta)
    assert torch.equal(C, C2)  # deterministic


@pytest.mark.gpu
def test_ops_refuse_host_tensors(cuda_device):
    """A host tensor handed to a kernel would fault the device; every op checks the
    devices of its tensor arguments on the host and raises instead."""
    from alphago_amd import ops

    ops.load()
    w = torch.randn(192, 64, 3, 3, device=cuda_device)
    wf_host = torch.zeros(9, 192, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="expected a GPU tensor"):
        ops.pack_weights([w], [wf_host])
    p = torch.zeros(1000, device=cuda_device)
    with pytest.raises(RuntimeError, match="expected a GPU tensor"):
        ops.sgd_update(p, torch.zeros(1000), 0.1)
    torch.cuda.synchronize()  # the device is still healthy
    assert float(p.sum()) == 0.0


@pytest.mark.parametrize("B,S", [(3, 19), (5, 9), (2, 13), (1, 8)])
@LAB
def test_winograd_lab_forward(ops, cuda_device, B, S):
    """Kernel-lab Winograd F(2x2,3x3) forward (winograd.hip) vs fp32 F.conv2d: odd and even board
    sizes (the last tile row/column of an odd board reads past the padded image: zero), tile counts
    that do not fill the last 32-tile workgroup, bias + ReLU, borders untouched."""
    torch.manual_seed(9)
    C = 192
    L = ops.lab()
    x = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w = torch.randn(C, C, 3, 3, device=cuda_device) * 0.05
    b = torch.randn(C, device=cuda_device) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    y = ops.padded_empty(B, S, 1, C, cuda_device)
    L.wino_fwd(ops.to_padded(x, 1), ops.wino_pack_weights(w), b, y, S)
    torch.cuda.synchronize()
    assert _rel_err(ops.from_padded(y, 1), ref) < 1.5e-2
    assert y[:, 0].abs().sum() == 0 and y[:, :, -1].abs().sum() == 0


@pytest.mark.parametrize("B", [1, 4, 16, 32, 64])
@pytest.mark.parametrize("tile,ring", [(0, "0"), (36, "0"), (37, "0"),
                                       pytest.param(0, "1", marks=LAB), pytest.param(65, "1", marks=LAB),
                                       pytest.param(130, "0", marks=LAB)])
def test_small_batch_conv_fwd_dgrad_wgrad(ops, cuda_device, B, tile, ring):
    """Small batches (the reference's -B 16 training and batch-1 search calls): forward with the
    bitmask, bitmask dgrad and the wgrad the trainer picks (ops.wgrad_config: per-tap splits, the
    small-batch 64 x 64 plan at B = 32 / 64) vs fp32
    conv2d / conv2d_input / conv2d_weight.  Lab cases: the LDS-ring tiles 65 / 130 and the ring wgrad
    (variant 9 with 16-stage splits), retired from the production library in round 5."""
    torch.manual_seed(12)
    S, C = 19, 192
    x = _bf(torch.randn(B, C, S, S, device=cuda_device))
    w = _bf(torch.randn(C, C, 3, 3, device=cuda_device) * 0.05)
    b = torch.randn(C, device=cuda_device) * 0.1
    wf = ops.packed_weight_like(w, C, C)
    wd = ops.packed_weight_like(w, C, C, True)
    ops.pack_weights([w.contiguous()], [wf], [wd])
    xp = ops.to_padded(x, 1)
    y = ops.padded_empty(B, S, 1, C, cuda_device)
    mb = torch.full((B * (S + 2) ** 2 * ops.mbits_words(C),), -1, dtype=torch.int32, device=cuda_device)
    _conv_fwd(ops, tile, xp, wf, b, y, 3, S, 1, 1, mbits=mb)
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    g = _bf(torch.randn(B, C, S, S, device=cuda_device))
    dx = ops.padded_empty(B, S, 1, C, cuda_device)
    _conv_fwd(ops, tile, ops.to_padded(g, 1), wd, None, dx, 3, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mb)
    var, ns = ops.wgrad_config(B * S * S, C, C, 3)
    assert (var == ops.WGRAD_SMALL) == (ops.WGRAD_SMALL_M[0] < B * S * S <= ops.WGRAD_SMALL_M[1])
    if ring == "1":  # the lab's ring wgrad: one workgroup per CU, 16 32-pixel stages per split
        taps, per_split, _, _ = ops.wgrad_plan(C, C, 3)
        var, ns = 9, max(1, min(256 // per_split, (B * S * S + 31) // 32 // 16))
    assert ns > 0
    slab = torch.full((ns, 9, C, C), float("nan"), device=cuda_device)
    dbs = torch.zeros(ns, C, device=cuda_device)
    ops.conv_wgrad(xp, ops.to_padded(g, 1), slab, dbs, 3, S, 1, 1, variant=var)
    gw = torch.zeros(C, C, 3, 3, device=cuda_device)
    gb = torch.zeros(C, device=cuda_device)
    ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)
    torch.cuda.synchronize()
    assert _rel_err(ops.from_padded(y, 1), ref) < 1e-2
    ref_dx = torch.nn.grad.conv2d_input((B, C, S, S), w, g, padding=1) * (ref > 0)
    assert _rel_err(ops.from_padded(dx, 1), ref_dx) < 1e-2
    assert _rel_err(gw, torch.nn.grad.conv2d_weight(x, (C, C, 3, 3), g, padding=1)) < 2e-3
    assert _rel_err(gb, g.sum(dim=(0, 2, 3))) < 2e-3


@pytest.mark.parametrize("B,S,Cin,Cout,K,ns", [(1, 19, 192, 192, 3, 9), (4, 19, 192, 192, 3, 3), (16, 19, 192, 192, 3, 3),
                                            (3, 19, 64, 192, 5, 8), (5, 13, 128, 128, 3, 4), (7, 9, 64, 64, 3, 2),
                                            (2, 19, 192, 192, 3, 1), (1, 19, 160, 160, 3, 7), (4, 19, 160, 160, 3, 3),
                                            (2, 19, 64, 160, 5, 8)])
def test_conv_fwd_splitk(ops, cuda_device, B, S, Cin, Cout, K, ns):
    """Split-K 32-pixel conv (tile 38: the K loop over ns workgroups per tile, fp32 partials, one
    finishing pass): forward with bias + ReLU + bitmask and the bitmask dgrad vs fp32 conv2d /
    conv2d_input, and its bitmask equal to the one-pass tile-36 kernel's (tile 64 at the 160 value
    width, whose 160 -> 160 layers run straddled K-steps) up to pre-activations that round across
    zero."""
    torch.manual_seed(21)
    P = K // 2
    x = _bf(torch.randn(B, Cin, S, S, device=cuda_device))
    w = _bf(torch.randn(Cout, Cin, K, K, device=cuda_device) * 0.05)
    b = torch.randn(Cout, device=cuda_device) * 0.1
    ref = F.relu(F.conv2d(x, w, b, padding=P))
    wf = ops.packed_weight_like(w, Cin, Cout)
    ops.pack_weights([w.contiguous()], [wf])
    xp = ops.to_padded(x, P, Cin)
    M = B * S * S
    ws = torch.full((ns * M * Cout,), float("nan"), device=cuda_device)
    words = ops.mbits_words(Cout)
    mb = torch.full((B * (S + 2) ** 2 * words,), -1, dtype=torch.int32, device=cuda_device)
    mb36 = mb.clone()
    y = ops.padded_empty(B, S, 1, Cout, cuda_device)
    y36 = ops.padded_empty(B, S, 1, Cout, cuda_device)
    ops.conv_fwd_splitk(xp, wf, b, y, K, S, P, 1, ops.MODE_BIAS_RELU, mb, ws, ns)
    ops.conv_fwd(xp, wf, b, y36, K, S, P, 1, mbits=mb36, tile=64 if Cout == 160 else 36)
    torch.cuda.synchronize()
    assert _rel_err(ops.from_padded(y, 1), ref) < 1e-2
    assert y[:, 0].abs().sum() == 0 and y[:, :, -1].abs().sum() == 0
    assert (mb != mb36).float().mean().item() < 1e-3
    if Cin != Cout or K != 3:
        return
    # bitmask dgrad through the same workspace (Cin == Cout: the transposed 3x3 pack)
    wd = ops.packed_weight_like(w, Cin, Cout, True)
    ops.pack_weights([w.contiguous()], [wf], [wd])
    g = _bf(torch.randn(B, Cout, S, S, device=cuda_device))
    dx = ops.padded_empty(B, S, 1, Cin, cuda_device)
    ops.conv_fwd_splitk(ops.to_padded(g, 1, Cout), wd, None, dx, 3, S, 1, 1, ops.MODE_MASKBITS, mb36, ws, ns)
    torch.cuda.synchronize()
    y36f = ops.from_padded(y36, 1)
    ref_dx = torch.nn.grad.conv2d_input((B, Cin, S, S), w, g, padding=1) * (y36f > 0)
    assert _rel_err(ops.from_padded(dx, 1), ref_dx) < 1e-2


@pytest.mark.lab
@pytest.mark.parametrize("S,B,Cin,Cout,Cout_p", [(19, 5, 48, 192, 192), (19, 3, 49, 152, 160), (9, 7, 48, 192, 192),
                                                 (13, 2, 49, 152, 160), (19, 1, 40, 128, 128)])
def test_conv_fwd_packed_taps_first_layer(ops, cuda_device, S, B, Cin, Cout, Cout_p):
    """Packed-tap first layer (conv_fwd_pk: 8-channel chunks of the real planes only, up to three taps per
    K-step) vs fp32 conv2d, and its ReLU' bitmask equal to the 64-channel kernel's."""
    torch.manual_seed(13)
    K, P = 5, 2
    x = torch.randint(0, 2, (B, Cin, S, S), device=cuda_device).float()  # binary planes, as the featurizer's
    w = _bf(torch.randn(Cout, Cin, K, K, device=cuda_device) * 0.05)
    b = torch.randn(Cout, device=cuda_device) * 0.1
    bp = torch.zeros(Cout_p, device=cuda_device)
    bp[:Cout] = b
    ref = F.relu(F.conv2d(x, w, b, padding=P))
    xp = ops.to_padded(x, P)
    assert ops.pk_shape_ok(Cin, xp.shape[3])
    wpk = ops.packed_weight_pk(w, Cout_p)
    wfull = ops.packed_weight_like(w, 64, Cout_p)
    ops.pack_weights([w.contiguous(), w.contiguous()], [wpk, wfull])
    words = ops.mbits_words(Cout_p)
    mb1 = torch.full((B * (S + 2) ** 2 * words,), -1, dtype=torch.int32, device=cuda_device)
    mb2 = mb1.clone()
    y = ops.padded_empty(B, S, 1, Cout_p, cuda_device)
    y2 = ops.padded_empty(B, S, 1, Cout_p, cuda_device)
    ops.conv_fwd_pk(xp, wpk, bp, y, K, S, P, 1, Cin, mbits=mb1)
    ops.conv_fwd(xp, wfull, bp, y2, K, S, P, 1, mbits=mb2)
    torch.cuda.synchronize()
    out = ops.from_padded(y, 1)[:, :Cout]
    assert _rel_err(out, ref) < 1e-2
    assert y[:, 0].abs().sum() == 0 and y[:, :, -1].abs().sum() == 0
    assert (ops.from_padded(y, 1)[:, Cout:] == 0).all()
    # same products in a different summation order: bf16 outputs within rounding, same signs
    assert _rel_err(ops.from_padded(y, 1), ops.from_padded(y2, 1)) < 1e-2
    diff = (mb1 != mb2).float().mean().item()
    assert diff < 1e-3, diff  # bits differ only where a pre-activation rounds across zero


@pytest.mark.parametrize("beta", [1.0, 2.0])
def test_sample_moves_distribution(ops, cuda_device, beta):
    """Fused sampler: draws follow probs ** beta (normalised), rows without a sensible move give -1,
    one-hot rows give their index, and a seed reproduces its draws."""
    torch.manual_seed(3)
    B, NP = 8192, 361
    base = torch.zeros(NP, device=cuda_device)
    base[[3, 50, 77, 200, 360]] = torch.tensor([0.1, 0.2, 0.3, 0.15, 0.25], device=cuda_device)
    probs = base.repeat(B, 1).contiguous()
    probs[0] = 0.0
    probs[0, 123] = 1.0
    has = torch.ones(B, dtype=torch.bool, device=cuda_device)
    has[1] = False
    out = ops.sample_moves(probs, has, beta, 11)
    again = ops.sample_moves(probs, has, beta, 11)
    other = ops.sample_moves(probs, has, beta, 12)
    torch.cuda.synchronize()
    assert torch.equal(out, again) and not torch.equal(out, other)
    assert out[0].item() == 123 and out[1].item() == -1
    rest = out[2:]
    assert set(rest.unique().tolist()) <= {3, 50, 77, 200, 360}
    w = base[[3, 50, 77, 200, 360]] ** beta
    expect = (w / w.sum()).cpu()
    got = torch.stack([(rest == i).float().mean() for i in (3, 50, 77, 200, 360)]).cpu()
    assert (got - expect).abs().max().item() < 0.02, (got, expect)
    # mask mode: the (B, NP) sensible-move mask instead of the flags -- same draws (row 1 all-zero)
    legal = (probs > 0).to(torch.uint8)
    legal[1] = 0
    legal[5, 0] = 1  # a sensible entry with zero probability does not change the draw
    via_mask = ops.sample_moves(probs, legal, beta, 11)
    torch.cuda.synchronize()
    assert torch.equal(via_mask, out)



@pytest.mark.parametrize("B,S,Cin,Cout,K", [(1, 19, 192, 192, 3), (4, 19, 192, 192, 3), (16, 19, 192, 192, 3),
                                            (33, 19, 192, 192, 3), (16, 19, 64, 192, 5), (3, 19, 64, 192, 5),
                                            (16, 19, 160, 160, 3), (2, 19, 160, 160, 3), (5, 9, 128, 128, 3),
                                            (7, 13, 64, 64, 3), (64, 19, 192, 192, 3), (4, 9, 192, 192, 3),
                                            (16, 13, 192, 192, 3), (64, 13, 160, 160, 3), (1, 9, 64, 192, 5)])
def test_conv_weight_stationary(ops, cuda_device, B, S, Cin, Cout, K):
    """Weight-stationary small-batch conv (tile 40, conv_ws.hip: a workgroup's output-channel slice held
    in VGPRs across its waves' K ranges, 16-pixel chunks streamed past): bias + ReLU forward vs fp32
    conv2d with its ReLU' bitmask equal to the 32-pixel tile's (up to pre-activations that round across
    zero), the bitmask dgrad vs conv2d_input, and no write outside the interior."""
    torch.manual_seed(40 + B)
    P = K // 2
    real = 48 if (Cin == 64 and K == 5) else (152 if Cin == 160 else Cin)
    oreal = 152 if Cout == 160 else Cout
    x = _bf(torch.randn(B, real, S, S, device=cuda_device))
    w = _bf(torch.randn(oreal, real, K, K, device=cuda_device) * 0.05)
    b = torch.randn(oreal, device=cuda_device) * 0.1
    bp = torch.zeros(Cout, device=cuda_device)
    bp[:oreal] = b
    ref = F.relu(F.conv2d(x, w, b, padding=P))
    wf = ops.packed_weight_like(w, Cin, Cout)
    ops.pack_weights([w.contiguous()], [wf])
    xp = ops.to_padded(x, P, Cin)
    words = ops.mbits_words(Cout)
    mb = torch.full((B * (S + 2) ** 2 * words,), -1, dtype=torch.int32, device=cuda_device)
    mb_ref = mb.clone()
    y = ops.padded_empty(B, S, 1, Cout, cuda_device)
    yr = ops.padded_empty(B, S, 1, Cout, cuda_device)
    wws = ops.ws_packed_like(wf)
    ops.ws_pack([wf], [wws])  # tile 40 reads the weight-stationary order
    ops.conv_fwd(xp, wws, bp, y, K, S, P, 1, mbits=mb, tile=40)
    ops.conv_fwd(xp, wf, bp, yr, K, S, P, 1, mbits=mb_ref, tile=64 if Cout == 160 else 36)
    torch.cuda.synchronize()
    out = ops.from_padded(y, 1)
    assert _rel_err(out[:, :oreal], ref) < 1e-2
    assert (out[:, oreal:] == 0).all()
    assert y[:, 0].abs().sum() == 0 and y[:, :, -1].abs().sum() == 0
    assert (mb != mb_ref).float().mean().item() < 1e-3
    if Cin != Cout or K != 3:
        return
    # bitmask dgrad (mode 3) with the transposed pack
    wd = ops.packed_weight_like(w, Cin, Cout, True)
    ops.pack_weights([w.contiguous()], [wf], [wd])
    wdws = ops.ws_packed_like(wd)
    ops.ws_pack([wd], [wdws])
    g = _bf(torch.randn(B, oreal, S, S, device=cuda_device))
    dx = ops.padded_empty(B, S, 1, Cin, cuda_device)
    ops.conv_fwd(ops.to_padded(g, 1, Cout), wdws, None, dx, 3, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mb_ref,
                 tile=40)
    torch.cuda.synchronize()
    yrf = ops.from_padded(yr, 1)[:, :real]
    ref_dx = torch.nn.grad.conv2d_input((B, real, S, S), w, g, padding=1) * (yrf > 0)
    dxo = ops.from_padded(dx, 1)
    assert _rel_err(dxo[:, :real], ref_dx) < 1e-2
    assert (dxo[:, real:] == 0).all()
