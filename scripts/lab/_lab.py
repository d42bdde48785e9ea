"""Shared helpers of the kernel-lab scripts: every experiment runs the
non-production kernels through the separately built lab library
(torch.ops.alphago_amd_lab, `python -m alphago_amd._build lab`) with explicit
tile / variant arguments -- the production library has no global switches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from alphago_amd import ops  # noqa: E402

TILE, STAMPS, WGV, FP8V = [0], [None], [0], [0]
FP8_OLD_TO_NEW = {0: 5, 1: 1, 2: 0, 3: 3, 4: 4}  # round-1 variant numbers -> ConvFp8Args::variant


def lab_conv_fwd(x, w, bias, y, K, S, Pin, Po=1, mode=0, mask=None, mbits=None):
    ops.lab().conv_fwd(x, w, bias, mask, y, K, S, Pin, Po, mode, mbits, TILE[0], STAMPS[0])
    return y


def lab_conv_wgrad(x, dz, slab, dbs, K, S, Pin, Po=1, cin_real=0):
    ops.lab().conv_wgrad(x, dz, slab, dbs, K, S, Pin, Po, cin_real, WGV[0])


def lab_conv_fwd_fp8(x8, w8, bias, scales, out_scale, K, S, Pin, Po=1, y_bf16=None, y_fp8=None, amax=None):
    ops.lab().conv_fwd_fp8(x8, w8, bias, scales, out_scale, amax, y_bf16, y_fp8, K, S, Pin, Po, FP8V[0])
