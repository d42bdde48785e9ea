"""Winograd F(2x2,3x3) for the benchmark layer, measured unfused with library pieces.

VERDICT r1 item 1 asks for Winograd on the 3x3 layers.  This probe prices its parts on the
MI355X with the fastest kernels available without writing a new one.  It uses the benchmark
layer: 192 -> 192 channels, 19x19 boards, batch 2176.

  direct      our conv_fwd_kernel (bias + ReLU, bf16 out)
  V-xform     input transform B^T d B -> V[16, B*100, C] bf16 (torch elementwise; its HBM bytes
              are the floor whatever kernel does it)
  GEMM        16 batched [B*100 x 192] x [192 x 192] bf16 GEMMs (hipBLASLt via torch.bmm), the
              Winograd multiply phase, from HBM
  GEMM-L2     the same GEMM shape on an L2-resident slab (M = 4096 per xi), repeated: the
              multiply phase's compute rate if the transforms were fused
  Y-xform     output transform A^T M A + bias + ReLU

Also checks the Winograd result against the fp32 direct conv.  Prints one JSON line.
"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from alphago_amd import ops  # noqa: E402

BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float32)
G = torch.tensor([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=torch.float32)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float32)


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / reps)
    return best * 1e6


def main():
    dev = torch.device("cuda")
    B, C, S = int(os.environ.get("WG_B", "2176")), 192, 19
    T = 10  # 10 x 10 tiles of 2 x 2 outputs (board padded to 20 x 20)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, C, S, S, device=dev, generator=g).relu_().bfloat16()
    w = (torch.randn(C, C, 3, 3, device=dev, generator=g) * (2.0 / (9 * C)) ** 0.5)
    bias = torch.randn(C, device=dev, generator=g) * 0.1

    # direct: our production kernel
    ops.load()
    xp = ops.to_padded(x.float(), 1, C)
    wp = ops.packed_weight_like(w, C, C)
    ops.pack_weights([w], [wp])
    yp = ops.padded_empty(B, S, 1, C, dev)
    t_direct = timeit(lambda: ops.conv_fwd(xp, wp, bias, yp, 3, S, 1))

    # Winograd pieces. d: [B, 22, 22, C] = the 19x19 board with a 1-pixel zero border and 2 more
    # zero columns/rows so that 10 tiles of stride 2 and width 4 fit.
    d = torch.zeros(B, 22, 22, C, device=dev, dtype=torch.bfloat16)
    d[:, 1:20, 1:20] = x.permute(0, 2, 3, 1)
    V = torch.empty(16, B * T * T, C, device=dev, dtype=torch.bfloat16)
    bt = BT.to(dev)

    def v_xform():
        p = d.unfold(1, 4, 2).unfold(2, 4, 2)  # [B, 10, 10, C, 4, 4]
        v = torch.einsum("ik,btucks,js->ijbtuc", bt, p.float(), bt)  # B^T d B
        V.copy_(v.reshape(16, B * T * T, C))

    U = torch.einsum("ik,ockl,jl->ijco", G.to(dev), w, G.to(dev)).reshape(16, C, C).bfloat16()
    M = torch.empty(16, B * T * T, C, device=dev, dtype=torch.bfloat16)

    def gemm():
        torch.bmm(V, U, out=M)

    m_l2 = 4096
    V2, M2 = V[:, :m_l2].contiguous(), M[:, :m_l2].contiguous()

    def gemm_l2():
        for _ in range(10):
            torch.bmm(V2, U, out=M2)

    at = AT.to(dev)
    Y = torch.empty(B, T * 2, T * 2, C, device=dev, dtype=torch.bfloat16)

    def y_xform():
        m = M.view(4, 4, B, T, T, C).float()
        y = torch.einsum("oi,ijbtuc,pj->btoupc", at, m, at)  # [B, 10, 2, 10, 2, C]
        Y.copy_((y.reshape(B, 20, 20, C) + bias).relu_())

    t_v = timeit(v_xform, 5)
    t_g = timeit(gemm)
    t_gl2 = timeit(gemm_l2) / 10
    t_y = timeit(y_xform, 5)

    # numerics vs the fp32 direct conv (interior 19 x 19)
    v_xform()
    gemm()
    y_xform()
    ref = F.conv2d(x.float(), w, bias, padding=1).relu_().permute(0, 2, 3, 1)
    win = Y[:, :19, :19].float()
    err = (win - ref).abs().max().item() / ref.abs().max().item()
    direct = yp[:, 1:20, 1:20].float()
    err_direct = (direct - ref).abs().max().item() / ref.abs().max().item()

    flop_direct = 2.0 * B * S * S * C * C * 9
    flop_gemm = 2.0 * 16 * B * T * T * C * C
    out = {
        "batch": B, "channels": C,
        "direct_us": round(t_direct, 1), "direct_tflops": round(flop_direct / t_direct / 1e6, 1),
        "v_xform_us": round(t_v, 1), "gemm_us": round(t_g, 1),
        "gemm_tflops": round(flop_gemm / t_g / 1e6, 1),
        "gemm_l2_us_full_size_equiv": round(t_gl2 * B * T * T / m_l2, 1),
        "gemm_l2_tflops": round(2.0 * 16 * m_l2 * C * C / t_gl2 / 1e6, 1),
        "y_xform_us": round(t_y, 1),
        "V_bytes_GB": round(V.numel() * 2 / 1e9, 2),
        "rel_err_winograd_bf16V": err, "rel_err_direct": err_direct,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
