"""HIP (gfx950) kernel library: loading + thin Python wrappers.

The kernels live in ``alphago_amd/csrc/kernels`` and are compiled in-tree into
``alphago_amd/_hip_kernels.so`` (``python -m alphago_amd._build hip``).  They
are registered as ``torch.ops.alphago_amd.*``.  There is no silent fallback:
``load()`` raises if the library is missing on a machine with a GPU.

Tensor conventions (see csrc/kernels/conv.hip): activations are zero-bordered
NHWC bf16 ``(B, S+2P, S+2P, C)`` with C a multiple of 64; packed conv weights
are bf16 ``(K*K, Cout_p, Cin_p)``.
"""
from __future__ import annotations

import os
import threading
from typing import Optional

import torch

from .. import _build

_lock = threading.Lock()
_loaded = False

MODE_BIAS_RELU, MODE_MASK, MODE_NONE, MODE_MASKBITS = 0, 1, 2, 3


def flavor() -> str:
    """Kernel library flavor: ``prod`` (default) or ``debug`` (device bounds
    checks, synchronising ops; ``ALPHAGO_AMD_KERNELS=debug``)."""
    f = os.environ.get("ALPHAGO_AMD_KERNELS", "prod")
    if f not in ("prod", "debug"):
        raise ValueError("ALPHAGO_AMD_KERNELS must be prod or debug")
    return f


def library_path() -> str:
    return _build.hip_path(flavor())


def load(build_if_missing: bool = True) -> None:
    """Load the HIP kernel library (building it first if it is absent)."""
    global _loaded
    if _loaded:
        return
    with _lock:
        if _loaded:
            return
        path = library_path()
        if not os.path.exists(path) or os.environ.get("ALPHAGO_AMD_REBUILD"):
            if not build_if_missing:
                raise RuntimeError("alphago_amd HIP kernels not built: %s" % path)
            _build.build_hip(flavor=flavor())
        torch.ops.load_library(path)
        _loaded = True


_lab_loaded = False


def lab():
    """The kernel-lab library (non-production conv tilings and variants) as
    ``torch.ops.alphago_amd_lab``; loads next to the production library."""
    global _lab_loaded
    load()
    with _lock:
        if not _lab_loaded:
            path = _build.hip_path("lab")
            if not os.path.exists(path):
                _build.build_hip(flavor="lab")
            torch.ops.load_library(path)
            _lab_loaded = True
    return torch.ops.alphago_amd_lab


def is_loaded() -> bool:
    return _loaded


def _ops():
    load()
    return torch.ops.alphago_amd


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def pad_filters(F: int) -> int:
    """Padded trunk width for the bf16 conv kernels: multiples of 64, except
    129..160 -> 160 (the value net's 152 filters, AlphaGo/models/value.py:7),
    which runs on 160-wide tiles with straddled K-steps instead of 192."""
    return 160 if 128 < F <= 160 else round_up(F, 64)


def conv_n_tile(C: int) -> int:
    """Output-channel tile of the conv kernels for C padded channels."""
    return 160 if C == 160 else 192 if C % 192 == 0 else 128 if C % 128 == 0 else 64


# ----------------------------------------------------------------- layout helpers
def padded_empty(B: int, S: int, P: int, C: int, device, dtype=torch.bfloat16) -> torch.Tensor:
    """Zero-initialised padded NHWC buffer (borders must stay zero)."""
    return torch.zeros((B, S + 2 * P, S + 2 * P, C), device=device, dtype=dtype)


def to_padded(x: torch.Tensor, P: int, Cp: Optional[int] = None) -> torch.Tensor:
    """NCHW (any float) -> zero-bordered NHWC bf16 with channels padded to Cp."""
    B, C, S, _ = x.shape
    Cp = Cp or round_up(C, 64)
    out = padded_empty(B, S, P, Cp, x.device)
    out[:, P:P + S, P:P + S, :C] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    return out


def from_padded(y: torch.Tensor, P: int, C: Optional[int] = None) -> torch.Tensor:
    """Zero-bordered NHWC -> NCHW fp32 interior."""
    S = y.shape[1] - 2 * P
    C = C or y.shape[3]
    return y[:, P:P + S, P:P + S, :C].permute(0, 3, 1, 2).float()


# ----------------------------------------------------------------- op wrappers
def conv_fwd(x, w_packed, bias, y, K: int, S: int, Pin: int, Po: int = 1, mode: int = MODE_BIAS_RELU, mask=None,
             mbits=None, tile: int = 0):
    """Conv + epilogue.  mode 0: bias + ReLU (mbits: also write the ReLU' bitmask);
    1: dgrad masked by ``mask`` > 0; 3: dgrad masked by the ``mbits`` bitmask.
    ``tile``: 0 = automatic, or a production tiling 128 / 256 / 384 / 385 (384 with the DMA issue
    spread through the MFMAs; the automatic choice for large batches)."""
    _ops().conv_fwd(x, w_packed, bias, mask, y, K, S, Pin, Po, mode, mbits, tile)
    return y


# split-K forward / dgrad (tile 38) below this many output pixels (B <= 8 at 19 x 19); ALPHAGO_AMD_SPLITK=0
# turns it off.  SL step (profiles/r4/README.md): B = 1 1.33k -> 1.74k positions/s, B = 4 5.3k -> 6.27k,
# B = 8 10.54k -> 11.09k; at B = 16 the count below is 1 (181 tiles already fill ~144 workgroups).
# Split count: ~144 workgroups per layer -- graph-timed 192 -> 192 3x3 forwards
# (scripts/r4/launch_floor.py) are fastest at 9 splits for B = 1 (11.4 us vs 16.8 unsplit), 6 for
# B = 2 and 3 for B = 4 (14.7 us; 9 splits 16.3): more splits cost more in partials than they hide
SPLITK_MAX_M = int(os.environ.get("ALPHAGO_AMD_SPLITK_MAX_M", "3000"))
SPLITK_TARGET_WGS = int(os.environ.get("ALPHAGO_AMD_SPLITK_WGS", "144"))


def splitk_nsplit(M: int, cout_p: int, cin_p: int, K: int, target_wgs: int = SPLITK_TARGET_WGS) -> int:
    """Split count of the small-batch split-K conv (conv_fwd_splitk): enough 32-pixel workgroups for
    ``target_wgs``, at least three K-steps (64-channel chunks of a tap; 160-channel inputs run
    straddled steps) per split; 1 = no split (large M, ALPHAGO_AMD_SPLITK=0)."""
    if M >= SPLITK_MAX_M or os.environ.get("ALPHAGO_AMD_SPLITK", "1") == "0":
        return 1
    tiles = (M + 31) // 32 * (cout_p // conv_n_tile(cout_p))
    nk = -(-K * K * cin_p // 64)
    return max(1, min(nk // 3, -(-target_wgs // tiles), 64))


# Weight-stationary small-batch conv (tile 40, conv_ws.hip): the output-channel slice's weights stay in
# the workgroup's VGPRs (read once, in the weight-stationary order of ws_pack) while 16-pixel chunks stream
# past through an LDS ring of input rows.  Automatic up to these output-pixel counts (graph-timed chains of
# 11 layers with distinct weights, scripts/r5/ws_bench.py, profiles/r5/README.md): 192-wide layers
# 6.7 / 9.8 / 12.6 / 18.7 us at B = 1 / 8 / 16 / 32 vs 20.3 / 19.4 / 19.9 / 22.6 on the automatic tile
# (30.1 vs 25.5 at B = 64), 160-wide 7.2 .. 16.7 us vs 20.1 .. 20.5.  Training steps stop at B = 16: there
# the forward and dgrad share the GPU with the side-stream wgrad, and the one-workgroup-per-CU kernel
# (122 KB of LDS) lost at B = 32 (SL 34.4k vs 36.2k positions/s; B = 16: 22.8k vs 22.0k, same box).
# ALPHAGO_AMD_WS=0: off.
WS_MAX_M = {192: 32 * 361, 160: 32 * 361}
WS_MAX_M_TRAIN = {192: 16 * 361, 160: 16 * 361}


def ws_pack(srcs, dsts) -> None:
    """Weight-stationary order (what conv_fwd tile 40 reads) of standard (T, Cout, Cin) bf16 packs into
    same-shape tensors, all pairs in one launch."""
    srcs, dsts = list(srcs), list(dsts)
    if srcs:
        _ops().ws_pack(srcs, dsts)


def ws_packed_like(w_packed: torch.Tensor) -> torch.Tensor:
    """A tensor for the weight-stationary copy of a standard bf16 pack (``ws_pack``)."""
    return torch.empty_like(w_packed)


def conv_ws_supported(cout_p: int, cin_p: int, K: int) -> bool:
    """Whether the weight-stationary kernel (tile 40) has an instantiation for this layer shape."""
    return bool(_ops().conv_ws_supported(cout_p, cin_p, K))


def ws_applies(M: int, cout_p: int, cin_p: int, K: int, training: bool = False) -> bool:
    """Whether a conv of M output pixels runs on the weight-stationary kernel (tile 40); ``training``:
    inside a training step (lower limit, see WS_MAX_M_TRAIN)."""
    limit = (WS_MAX_M_TRAIN if training else WS_MAX_M).get(conv_n_tile(cout_p), 0)
    if os.environ.get("ALPHAGO_AMD_WS", "1") == "0" or M > limit:
        return False
    return bool(_ops().conv_ws_supported(cout_p, cin_p, K))


def conv_fwd_splitk(x, w_packed, bias, y, K: int, S: int, Pin: int, Po: int, mode: int, mbits, ws, nsplit: int):
    """conv_fwd on the 32-pixel tile with its K loop split over ``nsplit`` workgroups per tile (fp32
    partials in ``ws``, >= nsplit * M * Cout floats) and one finishing pass: modes 0 (bias + ReLU,
    optional bitmask), 2 (none), 3 (bitmask dgrad)."""
    _ops().conv_fwd_splitk(x, w_packed, bias, y, K, S, Pin, Po, mode, mbits, ws, nsplit)
    return y


def sample_moves(probs: torch.Tensor, has: torch.Tensor, beta: float, seed: int,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B,) int64 device moves: one draw per board from probs ** beta (a counter-based hash of
    (seed, board) supplies the uniform), -1 where ``has`` is false (sample.hip).  ``has``: (B,) flags,
    or the (B, NP) uint8 sensible-move mask (the kernel reduces each row)."""
    if out is None:
        out = torch.empty(probs.shape[0], dtype=torch.int64, device=probs.device)
    _ops().sample_moves(probs.contiguous(), has.contiguous(), out, float(beta), int(seed) & ((1 << 63) - 1))
    return out


def pk_shape_ok(cin_real: int, cin_p: int) -> bool:
    """Whether the packed-tap forward (conv_fwd_pk) can run a first layer: 32 < cin_real < 64 real input
    channels in a 64-channel padded input (48 policy / 49 value planes)."""
    return cin_p == 64 and 32 < cin_real < 64




def packed_weight_pk(w_oihw: torch.Tensor, cout_p: int, device=None) -> torch.Tensor:
    """Zeroed packed-tap weights (ceil(K*K*cpt/8), Cout, 64), cpt = ceil(cin_real/8); pack_weights fills
    them (chunk j of step s = tap (8s + j) // cpt, channels 8 ((8s + j) % cpt) ..)."""
    K, cin = w_oihw.shape[2], w_oihw.shape[1]
    cpt = (cin + 7) // 8
    return torch.zeros(((K * K * cpt + 7) // 8, cout_p, 64), device=w_oihw.device if device is None else device,
                       dtype=torch.bfloat16)


def conv_fwd_pk(x, w_pk, bias, y, K: int, S: int, Pin: int, Po: int, cin_real: int, mbits=None):
    """Kernel lab: the first layer (bias + ReLU, optional ReLU' bitmask) on the packed-tap K loop -- only
    the cin_real real channels of the 64-channel padded input are multiplied (48 planes: 19 K-steps
    instead of 25).  It multiplies 24 % fewer MFMAs but a K-step's row gathers from two or three pixels,
    and at B = 2176 it measured 399.5 us against the 64-channel kernel's ~381-398 us (round 4), so the
    trainers no longer use it."""
    lab().conv_fwd_pk(x, w_pk, bias, y, K, S, Pin, Po, cin_real, mbits)
    return y


def mbits_words(cout_p: int) -> int:
    """32-bit ReLU'-bitmask words per padded pixel for a conv with cout_p output channels."""
    return cout_p // conv_n_tile(cout_p) * 8


def conv_wgrad(x, dz, slab, dbslab, K: int, S: int, Pin: int, Po: int = 1, cin_real: int = 0, variant: int = 0):
    """Split-K weight gradient into ``slab``; ``cin_real`` (< padded Cin) lets
    the kernel skip zero-padded input channels (only slab columns < cin_real are written).
    ``variant`` 0 = the production per-tap kernel; any other variant is a kernel-lab kernel
    (torch.ops.alphago_amd_lab: 9 = LDS ring, 10-13 = first-layer re-cuts, ...)."""
    (_ops() if variant in (0, WGRAD_SMALL) else lab()).conv_wgrad(x, dz, slab, dbslab, K, S, Pin, Po, cin_real,
                                                                  variant)


def conv_wgrad_reduce(slab, dbslab, grad_w, grad_b=None, scale: float = 1.0, beta: float = 0.0):
    _ops().conv_wgrad_reduce(slab, dbslab, grad_w, grad_b, scale, beta)


def conv_wgrad_reduce_multi(slabs, dbslabs, grad_ws, grad_bs, scale: float = 1.0, beta: float = 0.0):
    """Every listed layer's split-K reduce in ONE launch (<= 16 layers); bitwise equal to one
    ``conv_wgrad_reduce`` per layer (same fixed summation order)."""
    _ops().conv_wgrad_reduce_multi(list(slabs), list(dbslabs), list(grad_ws), list(grad_bs), float(scale),
                                   float(beta))


def conv_wgrad_direct(x, dz, grad_w, grad_b, K: int, S: int, Pin: int, Po: int = 1, scale: float = 1.0,
                      beta: float = 0.0, ksub: int = 4):
    """Split-free weight gradient (C++ kWgradDirect): every workgroup owns one 32 x 48 (or 32 x 32) tile of
    one tap over all B*S*S pixels and writes ``grad_w`` (OIHW fp32, real channel counts: grad_w.shape[1] <
    the padded Cin skips the zero planes) = beta * grad_w + scale * dW, and ``grad_b`` likewise -- no split
    slab, no reduce launch, deterministic.  ``ksub``: 32-pixel sub-steps per pipeline stage (1 / 2 / 4 / 8)."""
    _ops().conv_wgrad_direct(x, dz, grad_w, grad_b, K, S, Pin, Po, float(scale), float(beta), int(ksub))


def wgrad_direct_supported(cout_p: int, cin_p: int, cin_real: int, K: int) -> bool:
    return bool(_ops().wgrad_direct_supported(cout_p, cin_p, cin_real or cin_p, K))


def policy_head_train(y, w, b, target, dz, loss, correct, dhead, S: int, grad_scale: float, weight=None,
                      bce: bool = False):
    """Fused policy head training step; ``bce`` selects the reference RL loss
    (binary CE on the softmax, reinforcement_policy_trainer.py:109) instead of CE."""
    _ops().policy_head(y, w, b, target, None, weight, dz, loss, correct, dhead, None, S, grad_scale, 1.0,
                       1 if bce else 0)


def head_grad_sums(dhead, loss, correct, grad, sums):
    """grad = dhead.sum(0) and sums[:2] = (loss.sum(), correct.sum()) in one deterministic launch."""
    _ops().head_grad_sums(dhead, loss, correct, grad, sums)


def policy_head_probs(y, w, b, probs, S: int, legal=None, temperature: float = 1.0):
    _ops().policy_head(y, w, b, None, legal, None, None, None, None, None, probs, S, 0.0, temperature)
    return probs


def pack_input(planes_u8, out, P: int, sym=None, target=None, target_out=None, rows=None, out8=None):
    """uint8 planes -> padded NHWC bf16 with the per-board D4 symmetry ``sym`` (and the target moved
    with it).  ``rows`` (int64, B): board b is ``planes_u8[rows[b]]`` -- the minibatch gather from a
    resident pool fused into the pack (a row outside the pool packs an all-zero board).  ``out8``
    (uint8, out's shape): the same values as e4m3 too (``quantize_fp8(out, out8, 0)``'s bytes)."""
    _ops().pack_input(planes_u8, sym, target, target_out, out, P, rows, out8)
    return out


def pack_weights(ws, wf, wd=()):
    _ops().pack_weights(list(ws), list(wf), list(wd))


def comm_proxy(src, dst, channels: int, wire_us: float):
    """RCCL all-reduce stand-in on the current stream (csrc/kernels/comm_proxy.hip)."""
    _ops().comm_proxy(src, dst, channels, wire_us)


def sgd_update(p, g, lr: float, gscale: float = 1.0):
    _ops().sgd_update(p, g, lr, gscale)


OPT_SGD, OPT_MOMENTUM, OPT_ADAM = 0, 1, 2


def sgd_pack(p, g, lr: float, w_meta, wf, wd, ranges, sched=None, gscale: float = 1.0, opt: int = OPT_SGD,
             m1=None, m2=None, momentum: float = 0.0, beta_1: float = 0.9, beta_2: float = 0.999,
             epsilon: float = 1e-8, nesterov: bool = False):
    """Fused optimizer step + bf16 weight packs in one launch (pack.hip sgd_pack_kernel): conv layer i's
    weights at flat offset w_meta[i][0] with shape (Cout, Cin, K, K) = w_meta[i][1:]; the same update over
    ``ranges`` ((offset, length) pairs: biases, head); ``sched`` (device Keras schedule) replaces ``lr``.
    ``opt``: OPT_SGD, OPT_MOMENTUM (velocity ``m1``) or OPT_ADAM (moments ``m1``, ``m2``; ``lr`` is then the
    bias-corrected lr_t, or ``sched`` an 8-entry schedule that computes it) -- Keras 1.0 semantics."""
    meta = [int(v) for m in w_meta for v in m]
    _ops().sgd_pack(p, g, float(lr), sched, float(gscale), meta, list(wf), list(wd), [int(o) for o, _ in ranges],
                    [int(n) for _, n in ranges], int(opt), m1, m2,
                    [float(momentum), float(beta_1), float(beta_2), float(epsilon), 1.0 if nesterov else 0.0])


def dense_f32(A, B, C, bias=None, trans_a: bool = False, trans_b: bool = False, beta: float = 0.0):
    """C = beta*C + op(A) @ op(B) (+ bias) in exact fp32 on the f32 MFMA (value-head dense layers);
    op(X) = X.T when trans_* (read in place, no copies)."""
    _ops().dense_f32(A, B, bias, C, trans_a, trans_b, beta)
    return C


def ladder_planes(board, meta, out, S: int, budget: int = 0):
    """Ladder bits on the device from the compact encoding (board int8 (B, S*S),
    meta int32 (B, 2) {ko, player to move}): out uint8 (B, S*S), bit 0 = ladder
    capture, bit 1 = ladder escape -- the host encoder's ladder bits.  ``budget``:
    node visits per read (0 = the engine's current budget, as the CPU reader)."""
    if budget <= 0:
        from .._native import engine

        budget = engine().ladder_budget()
    lab().ladder_planes(board, meta, out, S, budget)  # kernel lab (ladder.hip: slower than the host reader)
    return out


def sgd_update_sched(p, g, sched, gscale: float = 1.0):
    """SGD with the Keras decay schedule on the device: sched = float64
    {lr0, decay, iterations, lr}; advances iterations (HIP-graph capturable)."""
    _ops().sgd_update_sched(p, g, sched, gscale)


def packed_weight_like(w_oihw: torch.Tensor, cin_p: int, cout_p: int, transposed: bool = False,
                       device=None) -> torch.Tensor:
    """Zeroed packed bf16 weights (K*K, Cout, Cin) -- transposed (K*K, Cin, Cout) for dgrad.  When the
    reduction width (Cin, or Cout for dgrad) is an odd multiple of 32 there is one extra all-zero tap:
    the straddled K-steps' last half reads it."""
    K = w_oihw.shape[2]
    red = cout_p if transposed else cin_p
    T = K * K + (1 if red % 64 == 32 else 0)
    shape = (T, cin_p, cout_p) if transposed else (T, cout_p, cin_p)
    return torch.zeros(shape, device=w_oihw.device if device is None else device, dtype=torch.bfloat16)


def wgrad_tap_group(cout_p: int, cin_p: int, K: int) -> int:
    """Kernel taps one wgrad workgroup covers (K for tap-merged 64-wide c tiles, else 1)."""
    return int(_ops().wgrad_tap_group(cout_p, cin_p, K))


def wgrad_plan(cout_p: int, cin_p: int, K: int, cin_real: int = 0, variant: int = 0):
    """(taps per workgroup, workgroups per split, resident workgroups per CU, threads per workgroup) of
    the wgrad kernel the production library runs for this layer."""
    t, w, c, th = _ops().wgrad_plan(cout_p, cin_p, cin_real, K, variant)
    return int(t), int(w), int(c), int(th)


WGRAD_MIN_STAGES = int(os.environ.get("ALPHAGO_AMD_WGRAD_MIN_STAGES", "8"))


def wgrad_nsplit(M: int, cout_p: int, cin_p: int, K: int, cin_real: int = 0, target_wgs: int = 0,
                 cus: int = 256, variant: int = 0) -> int:
    """Pixel splits of the production wgrad: one resident round of workgroups over ``cus`` CUs
    (``target_wgs`` > 0 overrides the workgroup count).  A second, partial round of workgroups costs
    30-70 % (profiles/r2_wgrad_variants.md), so the grid never exceeds one round."""
    _, per_split, per_cu, _ = wgrad_plan(cout_p, cin_p, K, cin_real, variant)
    target = target_wgs if target_wgs > 0 else cus * per_cu
    nks = (M + 31) // 32
    # at least WGRAD_MIN_STAGES 32-pixel stages per split: at small batches one resident round of
    # 3-stage splits spends its time writing a 75-MB slab that the reduce then reads back
    # (B = 16: 16.6 us wgrad + 16.3 us reduce per layer, profiles/r3_small_batch.md)
    return max(1, min(target // per_split, nks // WGRAD_MIN_STAGES if target_wgs <= 0 else nks))


# conv_wgrad's small-batch plan (C++ kWgradSmall): 64 x 64 output tiles with the kernel row's three taps
# merged -- 27 workgroups per pixel split of a 192 -> 192 layer instead of 9 -- on one resident round
# (two per CU).  SL positions/s, same box, per-tap plan -> small plan (profiles/r5/README.md): B = 24
# 30.5k -> 32.1k, B = 32 35.7k -> 39.9k, B = 48 45.0k -> 46.7k, B = 64 54.2k -> 58.3k; B <= 16 equal or
# mixed (22.0-22.8k either way), so it starts above 16 boards.
WGRAD_SMALL = 14
WGRAD_SMALL_M = (16 * 361, 64 * 361)  # (exclusive, inclusive) output-pixel range


def wgrad_config(M: int, cout_p: int, cin_p: int, K: int, cin_real: int = 0, target_wgs: int = 0, cus: int = 256,
                 variant: int = 0):
    """(variant, nsplit) of a layer's wgrad: the requested variant and wgrad_nsplit, or in the small-batch
    range (WGRAD_SMALL_M) the small-batch plan for the 3x3 layers of 64-multiple widths.  (Round 4's
    small-batch LDS-ring variant 9 and the first-layer variants 10-12 are kernel-lab kernels since
    round 5: measured slower or equal.)"""
    if (variant == 0 and WGRAD_SMALL_M[0] < M <= WGRAD_SMALL_M[1] and K == 3 and cout_p % 64 == 0 and
            cin_p % 64 == 0 and cout_p != 160 and (cin_real == 0 or cin_real == cin_p)):
        _, per_split, per_cu, _ = wgrad_plan(cout_p, cin_p, K, cin_real, WGRAD_SMALL)
        target = target_wgs if target_wgs > 0 else cus * per_cu
        nks = (M + 31) // 32
        return WGRAD_SMALL, max(1, min(target // per_split, nks // WGRAD_MIN_STAGES))
    return variant, wgrad_nsplit(M, cout_p, cin_p, K, cin_real, target_wgs, cus, variant)


def wgrad_splits(M: int, T: int, n_tiles: int = 1, target_wgs: int = 512) -> int:
    """Number of pixel splits so the wgrad grid has ~target_wgs workgroups."""
    nks = (M + 31) // 32
    s = max(1, target_wgs // max(1, T * n_tiles))
    return max(1, min(s, nks))


def featurize(board, ages, meta, fids, fplanes, S: int, ladder=None, planes=None, nhwc=None, P: int = 0,
              sensible=None, legal=None, overflow=None):
    """GPU featurizer (csrc/kernels/featurize.hip); see alphago_amd.ops.gpu_features."""
    _ops().featurize(board, ages, meta, ladder, list(fids), list(fplanes), planes, nhwc, sensible, legal, overflow, S, P)


def head_logits(y, w, b, z, S: int):
    """z (B, S*S) fp32 = 1x1 conv of the padded NHWC activation y (value-net head)."""
    _ops().head_logits(y, w, b, z, S)
    return z


def head_backward(y, w, dlogits, dz, dhead, S: int, dz8=None, dz8_scale=None, dz8_amax=None):
    """ReLU'-masked dY of a 1x1 head conv from dlogits, plus per-board [dW | db] partials.  With
    ``dz8`` (uint8, y's shape) dY goes out as e5m2 of bf16(dY) * dz8_scale[0] with max |bf16(dY)| into
    ``dz8_amax`` (int32[64]) -- the bytes quantize_bf8 would make -- and ``dz`` is not written."""
    _ops().head_backward(y, w, dlogits, dz, dhead, S, dz8, dz8_scale, dz8_amax)


def value_out(h, w2, b2, v, target=None, weight=None, loss=None, correct=None, dh=None, dout=None,
              grad_scale: float = 1.0):
    """v = tanh(h w2 + b2); with target: MSE loss, sign agreement, dh and per-board [dw2 | db2]."""
    _ops().value_out(h, w2, b2, target, weight, v, loss, correct, dh, dout, grad_scale)
    return v


# ----------------------------------------------------------------- fp8 (e4m3)
FP8_MAX = 448.0
FP8_AMAX_SLOTS = 64  # per-layer amax accumulator slots (kFp8AmaxSlots)


def fp8_amax_buffer(L: int, device) -> torch.Tensor:
    """(L, 64) int32 per-layer amax accumulators (float bits); amax of layer l = view(float32)[l].max()."""
    return torch.zeros((L, FP8_AMAX_SLOTS), dtype=torch.int32, device=device)


def fp8_exponent(amax: float, margin: int = 1) -> int:
    """Power-of-two scale exponent e so that amax * 2^e fits e4m3 with `margin` bits of headroom."""
    import math

    if not amax or amax <= 0 or not math.isfinite(amax):
        return 0
    return int(math.floor(math.log2(FP8_MAX / amax))) - margin


def fp8_nchunks(K: int, cin_p: int) -> int:
    """64-channel e4m3 weight chunks (even count); cin_p = 160 uses three chunks per tap."""
    n = K * K * ((cin_p + 63) // 64)
    return n + (n & 1)


def fp8_chunk_width(cin_p: int) -> int:
    """Channels per packed fp8 weight chunk: 32 for 160-channel reductions (the value width: five
    32-channel chunks per tap, no zero half; ALPHAGO_AMD_FP8_CW32=0 restores 64), else 64."""
    return 32 if cin_p == 160 and os.environ.get("ALPHAGO_AMD_FP8_CW32", "1") == "1" else 64


def fp8_weight_shape(K: int, cin_p: int, rows_p: int):
    """Shape of packed e4m3 weights reducing over cin_p channels (forward: input channels; transposed
    dgrad pack: output channels) with rows_p rows: (chunks, rows_p, chunk width); the chunk count
    covers K*K taps and is a multiple of the chunks per 128-K step."""
    cw = fp8_chunk_width(cin_p)
    per = 128 // cw
    n = K * K * ((cin_p + cw - 1) // cw)
    return ((n + per - 1) // per * per, rows_p, cw)


def pack_weights_fp8(w_oihw: torch.Tensor, cout_p: int, cin_p: int, exponent=None):
    """fp32 OIHW -> (uint8 e4m3 (nch, cout_p, 64) scaled by 2^e, e)."""
    w = w_oihw.detach().float().contiguous()
    if exponent is None:
        exponent = fp8_exponent(float(w.abs().max()), margin=0)
    out = torch.empty(fp8_weight_shape(w.shape[2], cin_p, cout_p), dtype=torch.uint8, device=w.device)
    _ops().pack_weights_fp8(w, out, float(2.0 ** exponent), None)
    return out, exponent


def pack_weights_fp8_into(w_oihw: torch.Tensor, out: torch.Tensor, scale_dev: torch.Tensor, transposed: bool = False):
    """Re-pack into an existing buffer with a device-resident scale (no host sync); ``transposed``:
    the dgrad weights (rows = input channels, chunks over output channels, taps flipped)."""
    _ops().pack_weights_fp8(w_oihw, out, 1.0, scale_dev, transposed)


def pack_weights_fp8_multi(ws, outs, scales_dev: torch.Tensor, layer, transposed):
    """Every fp8 weight pack of a repack in ONE launch: job i packs ws[i] into outs[i] with the device
    scale scales_dev[layer[i]]; transposed[i] selects the dgrad layout (rows = input channels,
    taps flipped)."""
    ws, outs, layer, transposed = list(ws), list(outs), [int(x) for x in layer], [int(bool(x)) for x in transposed]
    for i in range(0, len(ws), FP8_PACK_MAX_JOBS):  # the kernel's job table holds 48 entries
        j = i + FP8_PACK_MAX_JOBS
        _ops().pack_weights_fp8_multi(ws[i:j], outs[i:j], scales_dev, layer[i:j], transposed[i:j])


FP8_PACK_MAX_JOBS = 48  # kMaxFp8PackJobs (csrc/kernels/ops.cpp)


def conv_dgrad_bits_bf8(dz, wd, dx, mbits, dx8, scale, K: int, S: int, amax=None, tile: int = 0):
    """Bitmask dgrad (conv_fwd mode 3) that also writes dx8 = e5m2(dx * scale[0]) for the fp8 wgrad
    and folds max |dx| into ``amax`` (int32[64] float bits: the next step's delayed scale)."""
    _ops().conv_dgrad_bits_bf8(dz, wd, dx, mbits, dx8, scale, amax, K, S, tile)


def conv_wgrad_fp8(x8, dz8, slab, dbslab, xscale, gscale, gmul, K: int, S: int, Pin: int, Po: int = 1, amax=None):
    """fp8 weight gradient of a 160 -> 160 3x3 layer (conv_wgrad_fp8.hip): e4m3 x8 (E8M0 exponent
    xscale[0]) x e5m2 dz8 (gscale[0]; gmul[0] = its 2^e multiplier, undone in the bias sums) into the
    same split slab as conv_wgrad; reduce with conv_wgrad_reduce.  ``amax`` (int32[64]): max |dZ|
    from the e5m2 bytes (the next step's delayed scale)."""
    _ops().conv_wgrad_fp8(x8, dz8, slab, dbslab, xscale, gscale, gmul, K, S, Pin, Po, amax)


def wgrad_fp8_supported(cout_p: int, cin_p: int, K: int) -> bool:
    """Shapes the fp8 wgrad kernel covers (the value net's 160 -> 160 3x3 layers)."""
    return cout_p == 160 and cin_p == 160 and K == 3


def wgrad_fp8_nsplit(M: int, K: int = 3, target_wgs: int = 512) -> int:
    """Pixel splits of the fp8 wgrad (128-pixel steps, one 160 x 160 tile per tap and split,
    two workgroups per CU): one resident round."""
    nks = (M + 127) // 128
    return max(1, min(target_wgs // (K * K), nks))


def wino_pack_weights(w_oihw: torch.Tensor) -> torch.Tensor:
    """Kernel-lab Winograd F(2x2, 3x3) weights (winograd.hip): U = G g G^T per (cout, cin), bf16,
    packed [16 xi][Cin/32][Cout/16][64 lanes][8] so that one MFMA B fragment is one 16-B load per
    lane (lane -> cout 16 nb + lane % 16, cin 32 ks + 8 (lane // 16) + e)."""
    w = w_oihw.detach().float()
    cout, cin = w.shape[:2]
    g = torch.tensor([[1.0, 0.0, 0.0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.0, 1.0]], device=w.device)
    u = torch.einsum("ik,nckl,jl->ijnc", g, w, g).reshape(16, cout, cin)
    u = u.reshape(16, cout // 16, 16, cin // 32, 4, 8).permute(0, 3, 1, 4, 2, 5)
    return u.contiguous().to(torch.bfloat16)


def absmax_bf16(x, amax):
    """max |x| of a bf16 tensor folded into fp8 amax slots (int32 float bits, per-slot atomicMax)."""
    _ops().absmax_bf16(x, amax, amax.view(torch.float32))


def conv_dgrad_fp8(dz8, w8t, mask, scales, out_scale, K: int, S: int, y_bf16, y_fp8=None, amax=None):
    """fp8 dgrad: dx = conv(dz8 (e5m2, E8M0 scale scales[0]), w8t (transposed e4m3, scales[1]))
    masked by mask > 0 (bf16 activation of the layer below); bf16 y_bf16 and optional e5m2
    y_fp8 (x out_scale); amax accumulates max |dx|."""
    _ops().conv_dgrad_fp8(dz8, w8t, mask, scales, out_scale, amax, y_bf16, y_fp8, K, S)


def conv_dgrad_fp8_bits(dz8, w8t, mbits, scales, out_scale, K: int, S: int, y_bf16=None, y_fp8=None, amax=None):
    """fp8 dgrad of the fp8-wgrad value step (160 channels): dz8 e5m2 (the copy the previous dgrad
    wrote for the fp8 wgrad; MFMA scale scales[0]) x the transposed flipped e4m3 weights (scales[1]),
    ReLU' from the forward's bitmask ``mbits``; writes y_fp8 = e5m2(dx * out_scale[0]) and/or bf16
    y_bf16; ``amax`` accumulates max |dx|."""
    _ops().conv_dgrad_fp8_bits(dz8, w8t, mbits, scales, out_scale, amax, y_bf16, y_fp8, K, S)


def conv_dgrad_fp8_bf16(dz, w8t, mbits, scales, in_scale, K: int, S: int, dx, amax=None):
    """fp8 dgrad straight from the bf16 gradient: dz (padded NHWC bf16) is converted to e5m2 in
    registers as the kernel loads it (multiplier in_scale[0], MFMA E8M0 scale scales[0]), times the
    transposed flipped e4m3 weights (scales[1]); ReLU' from the forward's bitmask ``mbits``; bf16 dx;
    ``amax`` accumulates max |dx| (the next layer's gradient scale)."""
    _ops().conv_dgrad_fp8_bf16(dz, w8t, mbits, scales, in_scale, amax, dx, K, S)


def fp8_grad_scales(amax, gscales8, gosc, margin: int = 1):
    """Delayed e5m2 gradient scaling: gosc[l] = 2^e, gscales8[l, 0] = 127 - e from amax[l] (cleared)."""
    _ops().fp8_grad_scales(amax, gscales8, gosc, margin)


def quantize_bf8(x_bf16: torch.Tensor, out: torch.Tensor, scale_dev: torch.Tensor, amax: torch.Tensor):
    """e5m2 quantisation (x * scale_dev[0]) with max |x| accumulated into amax (int32[64])."""
    _ops().quantize_bf8(x_bf16, out, scale_dev, amax)
    return out


def quantize_fp8_dev(x_bf16: torch.Tensor, out: torch.Tensor, scale_dev: torch.Tensor, amax: torch.Tensor):
    """e4m3 quantisation (x * scale_dev[0]) with max |x| accumulated into amax (int32[64]): a bf16 layer's
    output as the next fp8 layer's input in the mixed-precision fp8 step."""
    _ops().quantize_fp8_dev(x_bf16, out, scale_dev, amax)
    return out


def bf8_to_float(t_u8: torch.Tensor, exponent: int = 0) -> torch.Tensor:
    """Decode e5m2 bytes (and undo a 2^exponent scale)."""
    return t_u8.view(torch.float8_e5m2).float() * (2.0 ** -exponent)


def fp8_weight_scales(ws, wscale, scales8):
    """Per-layer e4m3 weight exponents on the device: wscale[l] = 2^e_l, scales8[l, 1] = 127 - e_l."""
    _ops().fp8_weight_scales(list(ws), wscale, scales8)


def fp8_act_scales(amax, scales8, osc, margin: int = 1, max_drop: int = 0):
    """Delayed activation scaling from the per-layer output amax (also clears amax).  ``max_drop`` > 0:
    underflow guard -- each layer's exponent falls by at most that many binades per step (outliers of a
    sudden amax rise saturate instead of flushing the bulk of the activations to zero)."""
    _ops().fp8_act_scales(amax, scales8, osc, margin, max_drop)


def quantize_fp8(x_bf16: torch.Tensor, out: torch.Tensor, exponent: int):
    _ops().quantize_fp8(x_bf16, out, float(2.0 ** exponent))
    return out


def conv_fwd_fp8(x8, w8, bias, scales, out_scale, K: int, S: int, Pin: int, Po: int = 1, y_bf16=None, y_fp8=None,
                 amax=None, mbits=None, sr_seed=None):
    """fp8 conv + bias + ReLU.  scales: int32 device tensor {127 - e_x, 127 - e_w} (MFMA E8M0);
    out_scale: f32 device tensor [2^e_y] for the e4m3 output; amax: int32[64] running max slots (float bits);
    sr_seed: int32 device scalar -> the e4m3 output is stochastically rounded (training forward)."""
    _ops().conv_fwd_fp8(x8, w8, bias, scales, out_scale, amax, y_bf16, y_fp8, K, S, Pin, Po, mbits, sr_seed)


def fp8_to_float(t_u8: torch.Tensor, exponent: int = 0) -> torch.Tensor:
    """Decode e4m3 bytes (and undo a 2^exponent scale)."""
    return t_u8.view(torch.float8_e4m3fn).float() * (2.0 ** -exponent)
