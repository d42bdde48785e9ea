"""Training-step engines for the policy network.

``HipPolicyTrainer`` is the MI355X path.  One SL step (reference:
supervised_policy_trainer.py:199-213, Keras ``train_on_batch`` + SGD) is a
fixed sequence of hand-written kernels over preallocated buffers:

  pack_input (uint8 planes -> padded NHWC bf16, per-board D4 symmetry, targets)
  L x conv_fwd (implicit GEMM on MFMA, fused bias+ReLU)
  policy_head (1x1 conv + softmax + clipped CE + top-1 + head backward)
  for l = L..1:
     conv_wgrad(l) -> split slab -> reduce into the flat fp32 grad
        -> async RCCL all-reduce of the bucket once complete (RCCL's own stream)
     conv_fwd in dgrad mode (flipped weights, ReLU' mask fused)
  sgd (flat fp32 master) + pack_weights (bf16 forward and dgrad copies)

The gradient all-reduce of a bucket overlaps the remaining backward.  dgrad
and wgrad of a layer are independent; ``overlap=True`` runs the wgrad on a
second HIP stream, but on MI355X the two big-LDS kernels then split the CUs
and the step is slower (alternating A/B, scripts/overlap_ab.sh: SL 118.7k vs
120.3k, value 131.2k vs 136.8k positions/s), so large batches run serial.  For
B = 8 .. 256 (``overlap=None``, the default) the kernels leave CUs idle and the overlap wins
(SL B = 16 19.6k -> 22.3k positions/s, round 4).  Every
activation and gradient has its own buffer (HBM is plentiful: ~2 GB at
batch 512), so there are no cross-stream reuse hazards.

``TorchPolicyTrainer`` is the same step with torch autograd (fp32 numerics
oracle; CPU path for tests and the "32-filter 2-layer on CPU" config).
"""
from __future__ import annotations

import os
import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .. import ops
from ..utils.profiling import trace_range
from ..models.nets import PolicyNet, ValueNet
from ..parallel import dist as agdist

# The 8 D4 symmetries as flat-index permutations (numpy semantics of the
# reference BOARD_TRANSFORMATIONS, supervised_policy_trainer.py:71-80).
_SYM_FWD = [
    lambda n, x, y: (x, y),
    lambda n, x, y: (n - 1 - y, x),
    lambda n, x, y: (n - 1 - x, n - 1 - y),
    lambda n, x, y: (y, n - 1 - x),
    lambda n, x, y: (x, n - 1 - y),
    lambda n, x, y: (n - 1 - x, y),
    lambda n, x, y: (y, x),
    lambda n, x, y: (n - 1 - y, n - 1 - x),
]


def symmetry_tables(n: int, device=None) -> torch.Tensor:
    """(8, n*n) long: fwd[s][p] = index of point p after symmetry s."""
    t = torch.empty(8, n * n, dtype=torch.long)
    for s, f in enumerate(_SYM_FWD):
        for x in range(n):
            for y in range(n):
                ox, oy = f(n, x, y)
                t[s, x * n + y] = ox * n + oy
    return t.to(device) if device is not None else t


def apply_symmetry(planes: torch.Tensor, targets: Optional[torch.Tensor], sym: torch.Tensor, table: torch.Tensor):
    """Torch implementation of the per-sample D4 augmentation (oracle for pack_input)."""
    B, C, S, _ = planes.shape
    fwd = table[sym.long()]  # (B, S*S)
    inv = torch.argsort(fwd, dim=1)
    flat = planes.reshape(B, C, S * S)
    out = torch.gather(flat, 2, inv.unsqueeze(1).expand(B, C, S * S)).reshape(B, C, S, S)
    tout = None
    if targets is not None:
        tl = targets.long()
        tout = torch.where(tl >= 0, torch.gather(fwd, 1, tl.clamp_min(0).unsqueeze(1)).squeeze(1), tl)
    return out, tout


class FlatParams:
    """fp32 master parameters and gradients, each in ONE flat device buffer.

    Module parameters are re-bound to views of the flat buffer so the rest of
    PyTorch (save/load, eval) sees ordinary parameters."""

    def __init__(self, named: Sequence[Tuple[str, torch.nn.Parameter]], device):
        self.names = [n for n, _ in named]
        sizes = [p.numel() for _, p in named]
        total = (sum(sizes) + 3) // 4 * 4
        self.flat = torch.zeros(total, device=device, dtype=torch.float32)
        self.grad = torch.zeros(total, device=device, dtype=torch.float32)
        self.segments: Dict[str, Tuple[int, int]] = {}
        self.views: Dict[str, torch.Tensor] = {}
        self.grad_views: Dict[str, torch.Tensor] = {}
        off = 0
        for (name, p), n in zip(named, sizes):
            v = self.flat[off:off + n].view(p.shape)
            v.copy_(p.data.to(device))
            p.data = v
            self.segments[name] = (off, n)
            self.views[name] = v
            self.grad_views[name] = self.grad[off:off + n].view(p.shape)
            off += n
        self.numel = off


OPTIMIZERS = ("sgd", "momentum", "adam")


class KerasSGDSchedule:
    """Keras 1.0 optimizer step size: lr / (1 + decay * iterations) (``SGD(lr, decay)``, the reference's
    optimizer, supervised_policy_trainer.py:199).  ``optimizer="momentum"`` is Keras ``SGD(lr, momentum,
    decay, nesterov)``; ``"adam"`` is Keras ``Adam(lr, beta_1, beta_2, epsilon)``, whose step is the
    bias-corrected lr_t = lr sqrt(1 - beta_2^t) / (1 - beta_1^t), t = iterations + 1 (the decay factor
    applies to it as well; Keras 1.0 Adam has none, so keep decay 0 for parity)."""

    def __init__(self, lr: float, decay: float = 0.0, iterations: int = 0, optimizer: str = "sgd",
                 momentum: float = 0.0, nesterov: bool = False, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-8):
        if optimizer not in OPTIMIZERS:
            raise ValueError("optimizer must be one of %s" % (OPTIMIZERS,))
        if optimizer == "momentum" and not 0.0 <= momentum < 1.0:
            raise ValueError("momentum must be in [0, 1)")
        self.lr, self.decay, self.iterations = lr, decay, iterations
        self.optimizer, self.momentum, self.nesterov = optimizer, momentum, nesterov
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon

    @property
    def opt_code(self) -> int:
        return OPTIMIZERS.index(self.optimizer)

    @property
    def n_moments(self) -> int:
        """Flat fp32 state buffers the optimizer keeps (velocity; Adam's two moments)."""
        return {"sgd": 0, "momentum": 1, "adam": 2}[self.optimizer]

    def current(self) -> float:
        lr = self.lr / (1.0 + self.decay * self.iterations)
        if self.optimizer == "adam":
            t = self.iterations + 1.0
            lr = lr * math.sqrt(1.0 - math.pow(self.beta_2, t)) / (1.0 - math.pow(self.beta_1, t))
        return lr

    def advance(self) -> None:
        self.iterations += 1

    def kernel_kwargs(self) -> dict:
        """Optimizer arguments of ops.sgd_pack."""
        return dict(opt=self.opt_code, momentum=self.momentum, beta_1=self.beta_1, beta_2=self.beta_2,
                    epsilon=self.epsilon, nesterov=self.nesterov)


def optimizer_update_(p: torch.Tensor, g: torch.Tensor, state: List[torch.Tensor], sched: KerasSGDSchedule,
                      step: float) -> None:
    """The fused kernel's update (pack.hip opt_update) in torch fp32 ops, same operation order."""
    with torch.no_grad():
        if sched.optimizer == "sgd":
            p.sub_(g * step)
        elif sched.optimizer == "momentum":
            v = state[0]
            v.mul_(sched.momentum).sub_(g * step)
            if sched.nesterov:
                p.add_(v * sched.momentum - g * step)
            else:
                p.add_(v)
        else:
            m, v = state
            m.mul_(sched.beta_1).add_(g * (1.0 - sched.beta_1))
            v.mul_(sched.beta_2).add_(g * g * (1.0 - sched.beta_2))
            p.sub_(step * m / (v.sqrt() + sched.epsilon))


# automatic wgrad / dgrad stream overlap between these pixel counts per step (B = 17 .. 256 at 19 x 19;
# round 5: with the weight-stationary forward / dgrad at B <= 16 -- one 12-wave workgroup per CU -- the
# side-stream wgrad no longer finds idle CUs there: B = 8 12.1k overlapped vs 14.1k serial, B = 16 23.0k
# vs 23.4k; B = 32 40.0k vs 35.8k, profiles/r5/README.md)
OVERLAP_AUTO_MIN_PIXELS, OVERLAP_AUTO_MAX_PIXELS = 17 * 361, 256 * 361
# split-free wgrad (ops.conv_wgrad_direct) up to this many output pixels per step: per 192 -> 192 layer
# B = 1 7.8 vs 19.3 us (split-K + reduce), B = 4 16.9 vs 21.2, B = 8 27.1 vs 24.8, B = 16 48.6 vs 26.2
# (ksub 4; profiles/r6/raw/wgrad_direct_bench_v1.jsonl)
WGRAD_DIRECT_MAX_PIXELS = 4 * 361
# one merged split-K reduce launch per backward (HipConvTrainer merged_reduce) up to this many pixels
# off: slower at every batch measured (B = 16 / 32 / 64 / 128 / 2176: -4 / -10 / -4 / -7 / -0.6 %; the merged
# launch reads twelve cold slabs, profiles/r6/README.md); merged_reduce=True opts in
MERGED_REDUCE_MAX_PIXELS = 0


class HipConvTrainer:
    """MFMA conv-trunk training engine; subclasses provide the head."""

    def __init__(self, net, batch: int, lr: float = 0.003, decay: float = 0.0, device=None, bucket_mb: float = 4.0,
                 overlap: Optional[bool] = None, wgrad_target_wgs: int = 0, iterations: int = 0, precision: str = "bf16",
                 wgrad_priority: Optional[int] = None, conv_tile: int = 0, fp8_dgrad: Optional[bool] = None,
                 reduce_stream: Optional[bool] = None, wgrad_variant: Optional[int] = None,
                 fp8_wgrad: Optional[bool] = None, optimizer: str = "sgd", momentum: float = 0.0,
                 nesterov: bool = False, fp8_bf16_layers: Optional[Sequence[int]] = None,
                 wgrad_direct: Optional[bool] = None, wgrad_ksub: int = 4, fp8_scale_guard: int = 0,
                 merged_reduce: Optional[bool] = None):
        ops.load()
        self._rows = None  # pool rows of the current training forward (compute_grads(rows=...))
        # fp8 underflow guard: activation scale exponents fall by at most this many binades per step
        # (ops.fp8_act_scales max_drop; 0 = the plain one-step delayed scale, the default: SL at lr 0.05
        # over 5 seeds collapsed 3 times with a 1-binade guard vs once unguarded and once in bf16,
        # profiles/r6/README.md)
        self.fp8_scale_guard = int(fp8_scale_guard)
        # wgrad kernel: 0 = per-tap kernel (default), 5 = one-kernel-row wgrad (opt-in, slower so far)
        self.wgrad_variant = int(os.environ.get("ALPHAGO_AMD_WGRAD_VARIANT", "0")) if wgrad_variant is None \
            else int(wgrad_variant)
        self.conv_tile = conv_tile  # forward/dgrad tiling: 0 = automatic, or 128 / 256 / 384 / 385
        # kernel-lab A/B only: the 3x3 forwards and dgrads on a lab tiling of the lab library
        # (torch.ops.alphago_amd_lab), e.g. 5 = compact halo + ping-pong (profiles/r3_chunk_outer.md)
        self.lab_tile = int(os.environ.get("ALPHAGO_AMD_LAB_TILE", "0"))
        if precision not in ("bf16", "fp8"):
            raise ValueError("precision must be bf16 or fp8")
        self.precision = precision
        self.env = agdist.env()
        self.device = torch.device(device) if device is not None else self.env.device
        if self.device.type != "cuda":
            raise RuntimeError("%s needs a GPU device" % type(self).__name__)
        self.net = net.to(self.device)
        self.batch = batch
        self.sched = KerasSGDSchedule(lr, decay, iterations, optimizer=optimizer, momentum=momentum,
                                      nesterov=nesterov)
        self.fp8_bf16_layers = frozenset(int(l) for l in (fp8_bf16_layers or ()))
        if reduce_stream is None:
            reduce_stream = os.environ.get("ALPHAGO_AMD_REDUCE_STREAM", "0") == "1"
        if overlap is None and reduce_stream:
            overlap = False  # an explicit reduce stream is a serial-backward mode: it wins over the auto overlap
        if overlap is None:
            # automatic: the wgrad on a side stream beside the dgrad at small batches, where both
            # kernels leave CUs idle -- SL B = 16 19.6k -> 22.3k, B = 256 95.3k -> 99.4k positions/s --
            # and serial from B = 512 on (108.8k vs 107.0k) and at the bench batch
            # (profiles/r4/raw/overlap_small_batch_ab.txt); ALPHAGO_AMD_OVERLAP=0 keeps it serial
            # Below B = 8 the steps are ~0.6 ms and the two-stream step measured mixed (B = 1 +8 %,
            # B = 2 -9 %, B = 4 -13..+2 %; raw/auto_overlap_splitk_batches.txt): serial there
            px = batch * net.board * net.board
            overlap = (precision == "bf16" and OVERLAP_AUTO_MIN_PIXELS <= px <= OVERLAP_AUTO_MAX_PIXELS
                       and os.environ.get("ALPHAGO_AMD_OVERLAP", "auto") != "0")
        self.overlap = overlap
        self.comm_events = None  # list: record the all-reduce wait of each backward as (start, end) events
        tr = net.trunk
        self.S = net.board
        self.L = tr.layers
        self.K = list(tr.widths)
        self.C0 = tr.in_planes
        self.C0p = ops.round_up(self.C0, 64)
        self.F = tr.filters
        # 152 filters (value net) run on 160-wide tiles, bf16 and fp8
        self.Fp = ops.pad_filters(self.F)
        if self.F > 256:
            raise ValueError("head kernels support up to 256 filters")
        self.P0 = self.K[0] // 2
        named = []
        for l in range(self.L):
            named.append(("w%d" % l, tr.weights[l]))
            named.append(("b%d" % l, tr.biases[l]))
        head = self._head_named_params()
        self.head_names = [n for n, _ in head]
        self.fp = FlatParams(named + head, self.device)
        if self.env.distributed:
            agdist.broadcast_(self.fp.flat, 0)
        # optimizer state (momentum velocity / Adam moments), flat fp32 like the master weights
        self.opt_state = [torch.zeros_like(self.fp.flat) for _ in range(self.sched.n_moments)]
        dev, B, S = self.device, batch, self.S
        # unpadded filters: the kernels read the biases straight from the flat
        # master parameters (no per-step copies); padded: zero-tailed copies
        self._bias_alias = self.Fp == self.F
        self.bias_p = ([self.fp.views["b%d" % l] for l in range(self.L)] if self._bias_alias
                       else [torch.zeros(self.Fp, device=dev) for _ in range(self.L)])
        self.wf, self.wd = [], []
        for l in range(self.L):
            cin_p = self.C0p if l == 0 else self.Fp
            w = self.fp.views["w%d" % l]
            self.wf.append(ops.packed_weight_like(w, cin_p, self.Fp))
            self.wd.append(ops.packed_weight_like(w, cin_p, self.Fp, transposed=True) if l > 0
                           else torch.empty(0, device=dev, dtype=torch.bfloat16))
        # activations / gradients (zero borders are never written)
        self.X0 = ops.padded_empty(B, S, self.P0, self.C0p, dev)
        self.Y = [ops.padded_empty(B, S, 1, self.Fp, dev) for _ in range(self.L)]
        self.DZ = [ops.padded_empty(B, S, 1, self.Fp, dev) for _ in range(self.L)]
        # ReLU' bitmasks of Y[0..L-2], written by the forward epilogue and read
        # by the dgrad epilogue instead of the bf16 activations (12x fewer bytes)
        hw = B * (S + 2) * (S + 2) * ops.mbits_words(self.Fp)
        self.MBITS = [torch.zeros(hw, dtype=torch.int32, device=dev) for _ in range(self.L - 1)]
        self.loss = torch.zeros(B, device=dev)
        self.correct = torch.zeros(B, device=dev)
        M = B * S * S
        self.nsplit = []
        self.wgrad_var = []
        slab_max, db_max = 0, 0
        for l in range(self.L):
            cin_p = self.C0p if l == 0 else self.Fp
            T = self.K[l] ** 2
            # one resident round of wgrad workgroups (the kernel's own occupancy, ops.wgrad_plan); small
            # batches: the LDS-ring variant with longer splits (ops.wgrad_config)
            var, ns = ops.wgrad_config(M, self.Fp, cin_p, self.K[l], self.C0 if l == 0 else 0, wgrad_target_wgs,
                                       self._num_cus(), self.wgrad_variant)
            self.nsplit.append(ns)
            self.wgrad_var.append(var)
            slab_max = max(slab_max, ns * T * self.Fp * cin_p)
            db_max = max(db_max, ns * self.Fp)
        # split-free wgrad (ops.conv_wgrad_direct: whole pixel range per workgroup, OIHW gradient written
        # in the kernel, no slab and no reduce launch); automatic up to WGRAD_DIRECT_MAX_PIXELS, off with
        # the reduce stream (its slabs are the point) and for kernel-lab wgrad variants
        if wgrad_direct is None:
            wgrad_direct = M <= WGRAD_DIRECT_MAX_PIXELS
        self.wgrad_ksub = int(wgrad_ksub)
        self.wgrad_direct = [bool(wgrad_direct) and not reduce_stream and self.wgrad_variant in (0, ops.WGRAD_SMALL)
                             and ops.wgrad_direct_supported(self.Fp, self.C0p if l == 0 else self.Fp,
                                                            self.C0 if l == 0 else self.Fp, self.K[l])
                             for l in range(self.L)]
        # small batches (B <= 8, ops.SPLITK_MAX_M): forward and bitmask dgrad on the split-K 32-pixel tile
        # (ops.conv_fwd_splitk: the K loop of a tile over several workgroups, one finishing pass);
        # bf16 path with the automatic tiling only
        self.sk_fwd = [1] * self.L
        self.sk_dg = [1] * self.L
        if conv_tile == 0 and self.precision == "bf16" and not self.lab_tile:
            for l in range(self.L):
                cin_p = self.C0p if l == 0 else self.Fp
                self.sk_fwd[l] = ops.splitk_nsplit(M, self.Fp, cin_p, self.K[l])
                if l > 0:
                    self.sk_dg[l] = ops.splitk_nsplit(M, self.Fp, self.Fp, self.K[l])
        # small batches: the weight-stationary kernel (tile 40) where it applies, instead of split-K
        self.ws_fwd = [False] * self.L
        self.ws_dg = [False] * self.L
        if conv_tile == 0 and self.precision == "bf16" and not self.lab_tile:
            for l in range(self.L):
                cin_p = self.C0p if l == 0 else self.Fp
                if ops.ws_applies(M, self.Fp, cin_p, self.K[l], training=True):
                    self.ws_fwd[l], self.sk_fwd[l] = True, 1
                if l > 0 and ops.ws_applies(M, self.Fp, self.Fp, self.K[l], training=True):
                    self.ws_dg[l], self.sk_dg[l] = True, 1
        # their weights in the weight-stationary order (ops.ws_pack after every update, repack())
        self.wf_ws = [ops.ws_packed_like(self.wf[l]) if self.ws_fwd[l] else None for l in range(self.L)]
        self.wd_ws = [ops.ws_packed_like(self.wd[l]) if self.ws_dg[l] else None for l in range(self.L)]
        sk_max = max(self.sk_fwd + self.sk_dg)
        self._sk_ws = torch.empty(sk_max * M * self.Fp, device=dev) if sk_max > 1 else None
        # Split-K reduce on a side stream (serial backward only): the memory-bound reduce of
        # layer l runs beside dgrad(l) instead of between the two big conv kernels.  The
        # slabs are double-buffered by layer parity, so wgrad(l-1) never waits for
        # reduce(l); wgrad(l-2) waits for reduce(l) through an event.
        self.s_r = (torch.cuda.Stream(device=dev, priority=-1) if reduce_stream and not overlap else None)
        nslab = 2 if self.s_r is not None else 1
        self._slabs = [torch.empty(slab_max, device=dev) for _ in range(nslab)]
        self._dbslabs = [torch.zeros(db_max, device=dev) for _ in range(nslab)]
        self._slab_free = [None] * nslab  # event: the reduce that last read slab i has finished
        # wgrad stream at high priority (-1): its workgroups are dispatched ahead of the
        # concurrent dgrad's, so the wgrad/reduce/all-reduce chain of a layer finishes
        # earlier and less of it is left after the last dgrad (+0.9 % positions/s,
        # 3 alternating A/B pairs of 100 steps; ALPHAGO_AMD_WGRAD_PRIO=0 restores equal priority)
        if wgrad_priority is None:
            wgrad_priority = int(os.environ.get("ALPHAGO_AMD_WGRAD_PRIO", "-1"))
        self.s_w = torch.cuda.Stream(device=dev, priority=wgrad_priority) if overlap else None
        # buckets over the flat grad, segments in backward order (head first)
        h0 = self.fp.segments[self.head_names[0]][0]
        h1 = sum(self.fp.segments[n][1] for n in self.head_names)
        segs = [(h0, h1)]
        self._seg_layer = [None]
        for l in reversed(range(self.L)):
            ow, nw = self.fp.segments["w%d" % l]
            _, nb = self.fp.segments["b%d" % l]
            segs.append((ow, nw + nb))
            self._seg_layer.append(l)
        self.buckets = agdist.make_buckets(segs, int(bucket_mb * (1 << 20)), last_alone=True)
        self._bucket_after_layer = {}
        for bi, (_, _, ids) in enumerate(self.buckets):
            last = ids[-1]
            self._bucket_after_layer[self._seg_layer[last] if self._seg_layer[last] is not None else -1] = bi
        self.reducer = agdist.BucketAllReducer(self.fp.grad, self.buckets)
        # one-GPU contention proxy of the overlapped all-reduce (ALPHAGO_AMD_COMM_PROXY, world 1 only)
        self._proxy = agdist.CommProxy.from_env(self.fp.grad, self.buckets) if not self.env.distributed else None
        if self._proxy is not None:
            self.reducer = self._proxy
        # merged reduce (one process, small batches): every layer's wgrad keeps its own split slab and ONE
        # ops.conv_wgrad_reduce_multi launch after the backward sums them all (the same fixed order per
        # element as the per-layer reduce, so bitwise equal) instead of a reduce launch per layer.  Without
        # a gradient all-reduce to overlap nothing waits for an early reduce.
        if merged_reduce is None:
            merged_reduce = M <= MERGED_REDUCE_MAX_PIXELS
        self.merged_reduce = (bool(merged_reduce) and not self.env.distributed and self._proxy is None
                              and self.s_r is None and self.L <= 16)
        self._mslabs = [None] * self.L  # per-layer (slab, dbias slab), allocated at first use
        self._pending_reduce = []
        # ALPHAGO_AMD_DEFER_ALLREDUCE=1: launch every bucket after the backward instead of at its bucket
        # point (no overlap, no CU contention with the dgrad / wgrad kernels)
        self.defer_allreduce = os.environ.get("ALPHAGO_AMD_DEFER_ALLREDUCE", "0") == "1"
        if precision == "fp8":
            # fp8 forward (block-scaled MFMA) with bf16 activations kept for the
            # backward; per-tensor power-of-two scales, all device-side:
            # weights from their amax at every repack, activations delayed by
            # one step from the amax the fp8 kernels accumulate.
            L = self.L
            self.w8 = [torch.zeros(ops.fp8_weight_shape(self.K[l], self.C0p if l == 0 else self.Fp, self.Fp),
                                   dtype=torch.uint8, device=dev) for l in range(L)]
            self.wscale8 = torch.ones(L, device=dev)
            self.scales8 = torch.full((L, 2), 127, dtype=torch.int32, device=dev)
            # this step's activation exponents, kept for the fp8 wgrad: X8[l] was quantised with
            # them, while scales8[:, 0] already holds the next step's delayed exponents by then
            self.xscale8 = torch.full((L, 1), 127, dtype=torch.int32, device=dev)
            self.osc8 = torch.ones(L, device=dev)
            self.amax8 = ops.fp8_amax_buffer(L, dev)
            # ALPHAGO_AMD_FP8_SR=1: the training forward rounds its e4m3 activations stochastically
            # (v_cvt_sr_fp8_f32; a device seed advanced every step); evaluation keeps round-to-nearest
            self.fp8_sr = os.environ.get("ALPHAGO_AMD_FP8_SR", "0") == "1"
            self._sr_seed = torch.zeros(1, dtype=torch.int32, device=dev)
            self._train_fwd = False
            self.X08 = torch.zeros(self.X0.shape, dtype=torch.uint8, device=dev)
            self.Y8 = [torch.zeros(self.Y[0].shape, dtype=torch.uint8, device=dev) for _ in range(2)]
            self._fp8_calibrated = False
            # fp8 dgrad (opt-in): e5m2 gradients x transposed e4m3 weights; per-layer delayed
            # gradient scales from the max |dZ| of the previous step (the first step runs bf16
            # dgrads and calibrates them).  Round 3: the kernel reads the bf16 dZ and converts it to
            # e5m2 in registers (no quantisation pass, no e5m2 tensor), takes ReLU' from the
            # forward's bitmask, and the transposed packs ride the one batched repack launch.
            self.fp8_dgrad = bool(fp8_dgrad)  # resolved below once fp8_wgrad is known
            self.wd8 = [None] + [torch.zeros(ops.fp8_weight_shape(self.K[l], self.Fp, self.Fp), dtype=torch.uint8,
                                             device=dev) for l in range(1, L)]
            self.gscales8 = torch.full((L, 2), 127, dtype=torch.int32, device=dev)
            self.gosc8 = torch.ones(L, device=dev)
            self.gamax8 = ops.fp8_amax_buffer(L, dev)
            self._g8_calibrated = False
            # fp8 wgrad (160 -> 160 3x3 layers, conv_wgrad_fp8.hip): e4m3 inputs kept per layer (the
            # forward's e4m3 outputs instead of a two-buffer ring), e5m2 output gradients written by
            # the bitmask dgrad's epilogue (the head's by one quantise pass), delayed gradient scales
            # as the fp8 dgrad's.  Layer 0 (49 planes) keeps the bf16 wgrad.  On by default where it
            # applies (value net: 143 vs 201 us per layer at B = 1024, profiles/r3_fp8_wgrad.md);
            # ALPHAGO_AMD_FP8_WGRAD=0 keeps the bf16 wgrad.
            if fp8_wgrad is None:
                fp8_wgrad = os.environ.get("ALPHAGO_AMD_FP8_WGRAD", "1") == "1"
            self.fp8_wgrad = bool(fp8_wgrad) and all(
                ops.wgrad_fp8_supported(self.Fp, self.Fp, self.K[l]) for l in range(1, L))
            # per-layer precision: the layers in fp8_bf16_layers run their forward, dgrad and wgrad in bf16
            # (their weights are never quantised); the others stay on the fp8 kernels
            self._w8layers = (set(range(1, L)) - self.fp8_bf16_layers) if self.fp8_wgrad else set()
            # With the fp8 wgrad the dgrad reads the same e5m2 dZ copy and writes e5m2 for the layer
            # below (conv_dgrad_fp8_bits): the all-fp8 backward is the default there (value 12 x 152,
            # B = 1024: 156.3k -> 179.9k positions/s, profiles/r3_fp8_wgrad.md);
            # ALPHAGO_AMD_FP8_DGRAD=0 keeps the bf16 dgrad.  Elsewhere fp8 dgrad stays opt-in.
            if fp8_dgrad is None:
                fp8_dgrad = self.fp8_wgrad and os.environ.get("ALPHAGO_AMD_FP8_DGRAD", "1") == "1"
            self.fp8_dgrad = bool(fp8_dgrad)
            if self.fp8_wgrad:
                self.X8 = [None] + [torch.zeros(self.Y[0].shape, dtype=torch.uint8, device=dev) for _ in range(1, L)]
                self.DZ8 = [None] + [torch.zeros(self.DZ[0].shape, dtype=torch.uint8, device=dev) for _ in range(1, L)]
                self.nsplit8 = ops.wgrad_fp8_nsplit(M, 3)
                need = self.nsplit8 * 9 * self.Fp * self.Fp
                if need > self._slabs[0].numel():
                    self._slabs = [torch.empty(need, device=dev) for _ in self._slabs]
                if self.nsplit8 * self.Fp > self._dbslabs[0].numel():
                    self._dbslabs = [torch.zeros(self.nsplit8 * self.Fp, device=dev) for _ in self._dbslabs]
        else:
            self.fp8_wgrad = False
            self._w8layers = set()
        # Keras-SGD schedule mirrored on the device (float64 {lr0, decay, iterations, lr}) so that
        # the SGD step reads its learning rate from memory: the whole step is graph-capturable
        self._sched_dev = torch.zeros(8, dtype=torch.float64, device=dev)
        # fused SGD + bf16 packs (ops.sgd_pack); ALPHAGO_AMD_FUSED_UPDATE=0: sgd_update + pack_weights
        self._fused_update = os.environ.get("ALPHAGO_AMD_FUSED_UPDATE", "1") == "1"
        self._pack_plan = None
        self.use_graph = False
        self._graphs = None
        self._g_in = None
        self._init_head()
        self.repack()

    # ------------------------------------------------------------------ schedule / graphs
    def sync_schedule(self) -> None:
        """Copy the host schedule (lr, decay, iterations) to the device copy used by graph replays."""
        sc = self.sched
        self._sched_dev.copy_(torch.tensor([sc.lr, sc.decay, float(sc.iterations), 0.0, sc.beta_1, sc.beta_2,
                                            float(sc.opt_code), 0.0], dtype=torch.float64))

    def enable_graphs(self, on: bool = True) -> None:
        """Run ``step`` as HIP-graph replays (bf16, per-board weights not supported): the first
        call runs eagerly (loads code objects, sets kernel attributes), the second captures
        the step -- pack, forward, head, backward (wgrad on its stream), SGD, repack -- and
        every call replays it.  With world > 1 the gradient all-reduce runs eagerly between a
        forward/backward graph and an update graph.  Replays are bitwise identical to eager steps.
        The learning-rate schedule is read from its device copy (synced from ``self.sched`` at
        capture); changing ``sched.lr`` afterwards needs ``sync_schedule()``."""
        if on and self.precision != "bf16":
            raise ValueError("graph-captured steps support the bf16 trainer only")
        self.use_graph = on
        self._graphs = None
        self._g_in = None
        self._graph_warm = False
        if on:
            self.sync_schedule()

    # ------------------------------------------------------------------ head API
    def _head_named_params(self):
        raise NotImplementedError

    def _init_head(self):
        pass

    def _head_train(self, targets, gscale: float, weight) -> None:
        raise NotImplementedError

    # ------------------------------------------------------------------ helpers
    def repack(self, bf16: bool = True) -> None:
        """Device copies of the master weights the kernels read: padded biases, the bf16 packs (unless
        the fused update already wrote them: ``bf16=False``) and the fp8 packs."""
        if not self._bias_alias:
            torch._foreach_copy_([b[:self.F] for b in self.bias_p], [self.fp.views["b%d" % l] for l in range(self.L)])
        ws = [self.fp.views["w%d" % l] for l in range(self.L)]
        if bf16:
            ops.pack_weights(ws, self.wf, self.wd)
        # the weight-stationary copies of the small-batch layers (from the bf16 packs, however written)
        src = [self.wf[l] for l in range(self.L) if self.wf_ws[l] is not None]
        src += [self.wd[l] for l in range(self.L) if self.wd_ws[l] is not None]
        ops.ws_pack(src, [w for w in self.wf_ws + self.wd_ws if w is not None])
        if self.precision == "fp8":
            ops.fp8_weight_scales(ws, self.wscale8, self.scales8)
            # every e4m3 pack of the step (forward, and the transposed dgrad packs) in ONE launch
            # (round 2: 12 + 11 launches of pack_weights_fp8 per step)
            dg = list(range(1, self.L)) if self.fp8_dgrad else []
            ops.pack_weights_fp8_multi([ws[l] for l in range(self.L)] + [ws[l] for l in dg],
                                       self.w8 + [self.wd8[l] for l in dg], self.wscale8,
                                       list(range(self.L)) + dg, [0] * self.L + [1] * len(dg))
            if self.fp8_dgrad:
                self.gscales8[:, 1].copy_(self.scales8[:, 1])

    _head_wrote_e5m2 = False  # this step's head wrote DZ8[L-1] (and its amax) instead of the bf16 DZ[L-1]

    def _top_e5m2_fusable(self) -> bool:
        """The fp8 backward reads only the e5m2 copy of the head's dZ (fp8 wgrad and dgrad of the top
        layer, scales calibrated), so a head can write that copy directly."""
        return (self.precision == "fp8" and self.fp8_wgrad and self.fp8_dgrad and self._g8_calibrated
                and (self.L - 1) in self._w8layers)

    def _layer_in(self, l):
        return (self.X0, self.P0) if l == 0 else (self.Y[l - 1], 1)

    def forward_trunk(self, planes: torch.Tensor, sym=None, move_targets=None, target_out=None) -> None:
        # fp8 trunk: the pack writes the e4m3 input copy too (was a quantize_fp8 pass over X0)
        ops.pack_input(planes, self.X0, self.P0, sym=sym, target=move_targets, target_out=target_out,
                       rows=self._rows, out8=self.X08 if self.precision == "fp8" else None)
        if self.precision == "fp8":
            if not self._fp8_calibrated:
                self._fp8_calibrate()
            self._forward_fp8()
            return
        for l in range(self.L):
            self._fwd_layer(l, self.MBITS[l] if l < self.L - 1 else None)

    def _fwd_layer(self, l: int, mbits=None) -> None:
        """bf16 forward of layer l into Y[l]."""
        x, pin = self._layer_in(l)
        if self.lab_tile and self.K[l] == 3:
            ops.lab().conv_fwd(x, self.wf[l], self.bias_p[l], None, self.Y[l], 3, self.S, pin, 1, 0, mbits,
                               self.lab_tile)
        elif self.ws_fwd[l]:
            ops.conv_fwd(x, self.wf_ws[l], self.bias_p[l], self.Y[l], self.K[l], self.S, pin, 1, mbits=mbits,
                         tile=40)
        elif self.sk_fwd[l] > 1:
            ops.conv_fwd_splitk(x, self.wf[l], self.bias_p[l], self.Y[l], self.K[l], self.S, pin, 1,
                                ops.MODE_BIAS_RELU, mbits, self._sk_ws, self.sk_fwd[l])
        else:
            ops.conv_fwd(x, self.wf[l], self.bias_p[l], self.Y[l], self.K[l], self.S, pin, 1, mbits=mbits,
                         tile=self.conv_tile)

    def _forward_fp8(self) -> None:
        x8, pin = self.X08, self.P0  # e4m3 input written by forward_trunk's pack_input (exact: 0/1 planes)
        # all-fp8 backward (fp8 wgrad + dgrad): below the last layer nothing reads the bf16
        # activations (wgrad reads the e4m3 copies, dgrad the ReLU' bits), so only e4m3 is written
        # (the first, calibrating backward runs bf16 wgrads on these activations)
        e4m3_only = self.fp8_wgrad and self.fp8_dgrad and self._g8_calibrated
        sr = self._sr_seed if (self.fp8_sr and self._train_fwd) else None
        bfl = self.fp8_bf16_layers
        for l in range(self.L):
            last = l == self.L - 1
            nxt_bf = l + 1 in bfl  # the next layer reads this output in bf16
            y8 = None if (last or nxt_bf) else (self.X8[l + 1] if self.fp8_wgrad else self.Y8[l % 2])
            if l in bfl:  # bf16 layer: bf16 conv, then the e4m3 copy the next (fp8) layer reads
                self._fwd_layer(l, None if last else self.MBITS[l])
                if y8 is not None:
                    ops.quantize_fp8_dev(self.Y[l], y8, self.osc8[l:l + 1], self.amax8[l])
            else:
                keep_bf16 = last or nxt_bf or not e4m3_only
                ops.conv_fwd_fp8(x8, self.w8[l], self.bias_p[l], self.scales8[l], self.osc8[l:l + 1], self.K[l],
                                 self.S, pin, 1, y_bf16=self.Y[l] if keep_bf16 else None, y_fp8=y8,
                                 amax=self.amax8[l], mbits=None if last else self.MBITS[l], sr_seed=sr)
            x8, pin = y8, 1
        if sr is not None:
            self._sr_seed.add_(1)
        if self.fp8_wgrad:
            self.xscale8.copy_(self.scales8[:, 0:1])
        ops.fp8_act_scales(self.amax8, self.scales8, self.osc8, 1, self.fp8_scale_guard)  # next step's scales

    @torch.no_grad()
    def _fp8_calibrate(self) -> None:
        """First step: activation scales from a bf16 forward of this batch."""
        amax = []
        for l in range(self.L):
            self._fwd_layer(l)
            amax.append(self.Y[l].amax().float())
        self.amax8.zero_()
        self.amax8[:, 0].copy_(torch.stack(amax).view(torch.int32))
        ops.fp8_act_scales(self.amax8, self.scales8, self.osc8, 1)
        self._fp8_calibrated = True

    def _num_cus(self) -> int:
        try:
            return int(torch.cuda.get_device_properties(self.device).multi_processor_count)
        except Exception:  # noqa: BLE001 - a query failure keeps the MI355X default
            return 256

    def _wgrad_layer(self, l: int, red: bool = False) -> None:
        """wgrad(l) into a split slab, then the deterministic reduce into the flat grad (and
        the async all-reduce of a completed bucket when ``red``).  With the reduce stream the
        reduce and the all-reduce launch run there; the caller's stream goes on to dgrad(l)."""
        x, pin = self._layer_in(l)
        T = self.K[l] ** 2
        cin_p = x.shape[3]
        f8 = l in self._w8layers and self._g8_calibrated
        ns = self.nsplit8 if f8 else self.nsplit[l]
        i = l % len(self._slabs)
        slab = self._slabs[i][:ns * T * self.Fp * cin_p].view(ns, T, self.Fp, cin_p)
        dbs = self._dbslabs[i][:ns * self.Fp].view(ns, self.Fp)
        sr = self.s_r
        if sr is not None and self._slab_free[i] is not None:
            torch.cuda.current_stream(self.device).wait_event(self._slab_free[i])
        if self.merged_reduce and not (self.wgrad_direct[l] and not f8):
            # this layer's own slab; the reduce waits for the merged launch after the backward
            if self._mslabs[l] is None or self._mslabs[l][0].numel() < ns * T * self.Fp * cin_p:
                self._mslabs[l] = (torch.empty(ns * T * self.Fp * cin_p, device=self.device),
                                   torch.zeros(ns * self.Fp, device=self.device))
            sl, db = self._mslabs[l]
            slab = sl[:ns * T * self.Fp * cin_p].view(ns, T, self.Fp, cin_p)
            dbs = db[:ns * self.Fp].view(ns, self.Fp)
            if f8:
                ops.conv_wgrad_fp8(self.X8[l], self.DZ8[l], slab, dbs, self.xscale8[l], self.gscales8[l, 0:1],
                                   self.gosc8[l:l + 1], self.K[l], self.S, pin, 1,
                                   amax=self.gamax8[l] if l < self.L - 1 else None)
            else:
                ops.conv_wgrad(x, self.DZ[l], slab, dbs, self.K[l], self.S, pin, 1,
                               cin_real=self.C0 if l == 0 else 0, variant=self.wgrad_var[l])
            self._pending_reduce.append((slab, dbs, l))
            return
        if self.wgrad_direct[l] and not f8:  # split-free: the OIHW gradient straight from the kernel
            ops.conv_wgrad_direct(x, self.DZ[l], self.fp.grad_views["w%d" % l], self.fp.grad_views["b%d" % l],
                                  self.K[l], self.S, pin, 1, 1.0, 0.0, self.wgrad_ksub)
            if red and not self.defer_allreduce and l in self._bucket_after_layer:
                self.reducer.launch(self._bucket_after_layer[l])
            return
        if f8:  # e5m2 dZ x e4m3 X, dequantised by the MFMA's block scales
            # (its tap-0 workgroups also fold max |dZ| into the delayed-scale slots of layer l)
            ops.conv_wgrad_fp8(self.X8[l], self.DZ8[l], slab, dbs, self.xscale8[l], self.gscales8[l, 0:1],
                               self.gosc8[l:l + 1], self.K[l], self.S, pin, 1,
                               amax=self.gamax8[l] if l < self.L - 1 else None)
        else:
            ops.conv_wgrad(x, self.DZ[l], slab, dbs, self.K[l], self.S, pin, 1, cin_real=self.C0 if l == 0 else 0,
                           variant=self.wgrad_var[l])

        def reduce():
            ops.conv_wgrad_reduce(slab, dbs, self.fp.grad_views["w%d" % l], self.fp.grad_views["b%d" % l], 1.0, 0.0)
            if red and not self.defer_allreduce and l in self._bucket_after_layer:
                self.reducer.launch(self._bucket_after_layer[l])

        if sr is None:
            reduce()
            return
        sr.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(sr):
            reduce()
            self._slab_free[i] = sr.record_event()

    def backward_trunk(self, reduce: bool = True) -> None:
        """dZ[L-1] (and head grads) must be ready on the current stream.
        ``reduce=False`` leaves the local gradient (gradient accumulation: the
        caller all-reduces the sum once)."""
        main = torch.cuda.current_stream(self.device)
        red = reduce and (self.env.distributed or self._proxy is not None)
        if red and not self.defer_allreduce and -1 in self._bucket_after_layer:
            self.reducer.launch(self._bucket_after_layer[-1])
        w8 = self.fp8_wgrad and self._g8_calibrated
        if w8 and self.L - 1 in self._w8layers and not self._head_wrote_e5m2:
            # the head's dZ in e5m2 for wgrad(L-1), and its max |dZ| (the value head writes it itself)
            top = self.L - 1
            ops.quantize_bf8(self.DZ[top], self.DZ8[top], self.gosc8[top:top + 1], self.gamax8[top])
        for l in reversed(range(self.L)):
            if self.s_w is not None:
                ev = main.record_event()
                with torch.cuda.stream(self.s_w):
                    self.s_w.wait_event(ev)
                    self._wgrad_layer(l, red)
            else:
                self._wgrad_layer(l, red)
            if l > 0:
                if w8 and self.fp8_dgrad and l in self._w8layers:
                    # all-fp8 backward: the e5m2 dZ copy wgrad(l) read is also this dgrad's operand;
                    # the output goes out as e5m2 (wgrad(l-1) and dgrad(l-1) read it) and as bf16 only
                    # for the first layer's bf16 wgrad; its max |dx| comes from wgrad(l-1)'s bytes
                    f8out = l - 1 in self._w8layers
                    ops.conv_dgrad_fp8_bits(self.DZ8[l], self.wd8[l], self.MBITS[l - 1], self.gscales8[l],
                                            self.gosc8[l - 1:l], self.K[l], self.S,
                                            y_bf16=None if f8out else self.DZ[l - 1],
                                            y_fp8=self.DZ8[l - 1] if f8out else None,
                                            amax=None if f8out else self.gamax8[l - 1])
                elif w8 and l - 1 in self._w8layers:  # bitmask dgrad + the e5m2 copy wgrad(l-1) reads
                    ops.conv_dgrad_bits_bf8(self.DZ[l], self.wd[l], self.DZ[l - 1], self.MBITS[l - 1],
                                            self.DZ8[l - 1], self.gosc8[l - 1:l], self.K[l], self.S,
                                            tile=self.conv_tile)
                elif (self.precision == "fp8" and self.fp8_dgrad and self._g8_calibrated
                      and l not in self.fp8_bf16_layers):
                    # fp8 dgrad straight from the bf16 dZ: converted to e5m2 in the kernel's registers
                    # (delayed per-layer scale gosc8[l]), ReLU' from the forward's bitmask, bf16 dx
                    # whose max |dx| sets the next step's scale of layer l-1
                    if l == self.L - 1:  # the head's dZ: its max |dZ| for the next step's scale
                        ops.absmax_bf16(self.DZ[l], self.gamax8[l])
                    ops.conv_dgrad_fp8_bf16(self.DZ[l], self.wd8[l], self.MBITS[l - 1], self.gscales8[l],
                                            self.gosc8[l:l + 1], self.K[l], self.S, self.DZ[l - 1],
                                            amax=self.gamax8[l - 1])
                elif self.lab_tile and self.K[l] == 3:  # kernel-lab A/B (see __init__)
                    ops.lab().conv_fwd(self.DZ[l], self.wd[l], None, None, self.DZ[l - 1], 3, self.S, 1, 1,
                                       ops.MODE_MASKBITS, self.MBITS[l - 1], self.lab_tile)
                elif self.ws_dg[l]:  # small batches: weight-stationary bitmask dgrad
                    ops.conv_fwd(self.DZ[l], self.wd_ws[l], None, self.DZ[l - 1], self.K[l], self.S, 1, 1,
                                 mode=ops.MODE_MASKBITS, mbits=self.MBITS[l - 1], tile=40)
                elif self.sk_dg[l] > 1:  # small batches: split-K bitmask dgrad
                    ops.conv_fwd_splitk(self.DZ[l], self.wd[l], None, self.DZ[l - 1], self.K[l], self.S, 1, 1,
                                        ops.MODE_MASKBITS, self.MBITS[l - 1], self._sk_ws, self.sk_dg[l])
                else:  # ReLU' bitmask from the forward epilogue (bf16 and fp8 forwards write it)
                    ops.conv_fwd(self.DZ[l], self.wd[l], None, self.DZ[l - 1], self.K[l], self.S, 1, 1,
                                 mode=ops.MODE_MASKBITS, mbits=self.MBITS[l - 1], tile=self.conv_tile)
        # join the side streams first: the fp8 wgrads still running there read gscales8 / gosc8
        # and fold max |dZ| into gamax8, which the scale update below rewrites and clears
        if self.s_w is not None:
            main.wait_stream(self.s_w)
        if self.s_r is not None:
            main.wait_stream(self.s_r)
        if self._pending_reduce:  # merged reduce: every deferred layer's split slab in one launch
            pr = self._pending_reduce
            ops.conv_wgrad_reduce_multi([p[0] for p in pr], [p[1] for p in pr],
                                        [self.fp.grad_views["w%d" % p[2]] for p in pr],
                                        [self.fp.grad_views["b%d" % p[2]] for p in pr], 1.0, 0.0)
            self._pending_reduce = []
        if self.precision == "fp8" and (self.fp8_dgrad or self.fp8_wgrad):
            if self._g8_calibrated:
                ops.fp8_grad_scales(self.gamax8, self.gscales8, self.gosc8, 1)  # next step's gradient scales
            else:
                self._fp8_grad_calibrate()
        if red:
            if self.defer_allreduce:
                for bi in range(len(self.buckets)):
                    self.reducer.launch(bi)
            if self.comm_events is not None:  # exposed all-reduce time (utils.metrics.StepMetrics)
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(main)
            self.reducer.wait()
            if self.comm_events is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(main)
                self.comm_events.append((e0, e1))

    @torch.no_grad()
    def _fp8_grad_calibrate(self) -> None:
        """First backward (bf16 dgrads): e5m2 scales of dZ_1..dZ_{L-1} from this step's max |dZ|."""
        amax = torch.stack([self.DZ[l].abs().amax().float() for l in range(self.L)])
        self.gamax8.zero_()
        self.gamax8[:, 0].copy_(amax.view(torch.int32))
        ops.fp8_grad_scales(self.gamax8, self.gscales8, self.gosc8, 1)
        self._g8_calibrated = True

    def compute_grads(self, planes: torch.Tensor, targets: torch.Tensor, sym: Optional[torch.Tensor] = None,
                      weight: Optional[torch.Tensor] = None, reduce: bool = True,
                      rows: Optional[torch.Tensor] = None):
        """Forward + backward into self.fp.grad (all-reduced when distributed,
        unless ``reduce=False``).  ``rows`` (int64, B): the minibatch is ``planes[rows]`` of a
        device-resident pool, gathered by the input-pack kernel itself (no separate index_select);
        ``targets``, ``sym`` and ``weight`` stay per board."""
        B = planes.shape[0] if rows is None else rows.numel()
        if B != self.batch:
            raise ValueError("batch %d != configured %d" % (B, self.batch))
        with trace_range("forward"):
            self._train_fwd = True
            self._rows = rows
            try:
                self._forward_for_head(planes, targets, sym)
            finally:
                self._train_fwd = False
                self._rows = None
        with trace_range("head"):
            self._head_train(targets, 1.0 / (B * self.env.world_size), weight)
        with trace_range("backward+allreduce"):
            self.backward_trunk(reduce)

    def _sgd_pack_plan(self):
        """(per-layer (flat offset, Cout, Cin, K, K), plain SGD ranges) of the fused update."""
        meta, wsegs = [], set()
        for l in range(self.L):
            off, n = self.fp.segments["w%d" % l]
            w = self.fp.views["w%d" % l]
            meta.append((off, w.shape[0], w.shape[1], w.shape[2]))
            wsegs.add(off)
        ranges = []
        for name in self.fp.names:
            off, n = self.fp.segments[name]
            if off in wsegs:
                continue
            if ranges and ranges[-1][0] + ranges[-1][1] == off:
                ranges[-1] = (ranges[-1][0], ranges[-1][1] + n)
            else:
                ranges.append((off, n))
        return meta, ranges

    def apply_update(self, device_schedule: bool = False) -> None:
        with trace_range("sgd+repack"):
            if self._fused_update:
                # one launch: SGD over the flat master weights + the bf16 forward / dgrad packs
                if self._pack_plan is None:
                    self._pack_plan = self._sgd_pack_plan()
                meta, ranges = self._pack_plan
                sched = None
                if device_schedule:  # the SGD kernels read the 4-entry prefix, Adam all 8
                    sched = self._sched_dev if self.sched.optimizer == "adam" else self._sched_dev[:4]
                st = self.opt_state
                ops.sgd_pack(self.fp.flat, self.fp.grad, 0.0 if device_schedule else self.sched.current(), meta,
                             self.wf, self.wd, ranges, sched=sched, m1=st[0] if st else None,
                             m2=st[1] if len(st) > 1 else None, **self.sched.kernel_kwargs())
                self.sched.advance()
                self.repack(bf16=False)
                return
            if self.sched.optimizer != "sgd":
                raise ValueError("momentum / Adam run in the fused update only (ALPHAGO_AMD_FUSED_UPDATE=1)")
            if device_schedule:
                # graph replays: lr = lr0 / (1 + decay * t) evaluated on the device (the same f64
                # expression as KerasSGDSchedule.current()) from the copy synced at capture time
                ops.sgd_update_sched(self.fp.flat, self.fp.grad, self._sched_dev[:4], 1.0)
            else:
                ops.sgd_update(self.fp.flat, self.fp.grad, self.sched.current(), 1.0)
            self.sched.advance()
            self.repack()

    def step(self, planes: torch.Tensor, targets: torch.Tensor, sym: Optional[torch.Tensor] = None,
             weight: Optional[torch.Tensor] = None, rows: Optional[torch.Tensor] = None):
        """One SGD step.  Returns (sum of per-board loss, metric sum) as device scalars (local;
        in graph mode static tensors, valid until the next step).  ``rows``: see compute_grads
        (eager steps only)."""
        if self.use_graph and weight is None:
            if rows is not None:
                raise ValueError("graph mode: pass the gathered minibatch, not pool rows")
            return self._graph_step(planes, targets, sym)
        self.compute_grads(planes, targets, sym, weight, rows=rows)
        self.apply_update()
        return self._step_metrics()

    def _step_metrics(self):
        return self.loss.sum(), self.correct.sum()

    def static_inputs(self, planes: torch.Tensor, targets: torch.Tensor, sym: Optional[torch.Tensor] = None):
        """Graph mode: the captured step's input buffers (allocated like the given tensors on first
        use).  A data pipeline that writes a batch straight into them (``index_select(out=...)``, a
        host copy) and passes them to ``step`` saves the step's three input copies."""
        if self._g_in is None:
            self._g_in = (torch.empty_like(planes), torch.empty_like(targets),
                          None if sym is None else torch.empty_like(sym))
            self._g_out = (torch.zeros((), device=self.device), torch.zeros((), device=self.device))
        return self._g_in

    def _graph_step(self, planes, targets, sym):
        gp, gt, gs = self.static_inputs(planes, targets, sym)
        if (sym is None) != (gs is None) or planes.shape != gp.shape:
            raise ValueError("graph mode: inputs must keep their shape and symmetry argument")
        if planes.data_ptr() != gp.data_ptr():  # the caller's own buffers: copy into the static ones
            gp.copy_(planes, non_blocking=True)
        if targets.data_ptr() != gt.data_ptr():
            gt.copy_(targets, non_blocking=True)
        if gs is not None and sym.data_ptr() != gs.data_ptr():
            gs.copy_(sym, non_blocking=True)
        # ALPHAGO_AMD_GRAPH_ALLREDUCE=1: the bucketed async all-reduce is captured inside the graph
        # (launched at its bucket points on RCCL's stream, joined before the update), so a graph step
        # keeps the eager step's overlap; by default the all-reduce runs eagerly between two graphs
        cap_ar = self.env.distributed and os.environ.get("ALPHAGO_AMD_GRAPH_ALLREDUCE", "0") == "1"
        dist = self.env.distributed and not cap_ar

        def grads():
            self.compute_grads(gp, gt, gs, None, reduce=not dist)

        def update():
            self.apply_update(device_schedule=True)
            l, c = self._step_metrics()  # the eager step's sums (same summation order: bitwise equal)
            self._g_out[0].copy_(l)
            self._g_out[1].copy_(c)

        if self._graphs is None:
            if not self._graph_warm:  # eager first step: code objects loaded, LDS attributes set
                self.sync_schedule()
                grads()
                if dist:
                    agdist.all_reduce_sum_(self.fp.grad)
                update()
                self._graph_warm = True
                return self._g_out
            torch.cuda.synchronize(self.device)
            self.sync_schedule()  # the device schedule continues from the host counter
            parts = [grads, update] if dist else [lambda: (grads(), update())]
            self._graphs = []
            # the wgrad side stream is captured as a parallel branch only on request
            # (ALPHAGO_AMD_GRAPH_OVERLAP=1); by default the graph is one serial chain
            keep_sw, keep_sr = self.s_w, self.s_r
            self.s_r = None  # captured serially: its slab events were recorded outside the capture
            if os.environ.get("ALPHAGO_AMD_GRAPH_OVERLAP", "0") != "1":
                self.s_w = None
            try:
                for fn in parts:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, capture_error_mode="thread_local"):
                        fn()
                    self._graphs.append(g)
            finally:
                self.s_w, self.s_r = keep_sw, keep_sr
            # the capture ran nothing; the iteration counters it advanced on the host are undone
            self.sched.iterations -= 1
        self._graphs[0].replay()
        if dist:
            agdist.all_reduce_sum_(self.fp.grad)
            self._graphs[1].replay()
        self.sched.advance()
        return self._g_out


class HipPolicyTrainer(HipConvTrainer):
    """Policy net: fused HIP head (softmax + clipped CE + top-1 + backward).
    ``weight`` (per board) scales each board's gradient — REINFORCE rewards."""

    def _head_named_params(self):
        return [("head_w", self.net.head_w), ("head_b", self.net.head_b)]

    def _init_head(self):
        self.dhead = torch.zeros(self.batch, self.F + 1, device=self.device)
        self.tgt = torch.zeros(self.batch, dtype=torch.int32, device=self.device)

    def _forward_for_head(self, planes, targets, sym):
        self.forward_trunk(planes, sym, targets, self.tgt)

    policy_loss = "ce"  # or "bce": the reference RL loss (binary CE on the softmax)

    def _head_train(self, targets, gscale, weight):
        hw = self.fp.views["head_w"].view(-1)
        hb = self.fp.views["head_b"]
        ops.policy_head_train(self.Y[-1], hw, hb, self.tgt, self.DZ[-1], self.loss, self.correct, self.dhead,
                              self.S, gscale, weight=weight, bce=self.policy_loss == "bce")
        ho, hn = self.fp.segments["head_w"]
        # head gradient and the step's two metric sums in one launch (a fresh 2-vector per step, so
        # the returned scalars stay valid after the next step)
        self._metric_sums = torch.empty(2, device=self.device)
        ops.head_grad_sums(self.dhead, self.loss, self.correct, self.fp.grad[ho:ho + hn + 1], self._metric_sums)

    def _step_metrics(self):
        return self._metric_sums[0], self._metric_sums[1]

    @torch.no_grad()
    def evaluate(self, planes: torch.Tensor, targets: torch.Tensor):
        """Loss/accuracy without update (validation)."""
        self.forward_trunk(planes, None, targets, self.tgt)
        hw = self.fp.views["head_w"].view(-1)
        ops.policy_head_train(self.Y[-1], hw, self.fp.views["head_b"], self.tgt, self.DZ[-1], self.loss,
                              self.correct, self.dhead, self.S, 0.0)
        return self.loss.sum(), self.correct.sum()


class HipValueTrainer(HipConvTrainer):
    """Value net (reference value.py:12-31): HIP trunk + 1x1 conv -> Dense(256)
    -> Dense(1) -> tanh head; MSE against game outcomes in [-1, 1].

    Head forward: ``head_logits`` (one pass over the last activation) -> z
    (B, 361) fp32; the 361x256 dense layer on the hand-written fp32 MFMA GEMM
    (``dense_f32``, csrc/kernels/dense.hip); ``value_out`` fuses the 256->1
    layer, tanh, MSE, sign accuracy and its backward.  Head backward:
    dz = dh W1^T and dW1 = z^T dh (the same kernel, operands read transposed
    in place, dW1 written straight into the flat gradient buffer), then
    ``head_backward`` writes the ReLU'-masked gradient into the MFMA trunk
    backward plus per-board partials of the 1x1 conv weight/bias.
    ``correct`` counts sign(v) == sign(z)."""

    def _head_named_params(self):
        n = self.net
        return [("head_w", n.head_w), ("head_b", n.head_b), ("fc1_w", n.fc1_w), ("fc1_b", n.fc1_b),
                ("fc2_w", n.fc2_w), ("fc2_b", n.fc2_b)]

    def _init_head(self):
        B, NP, dev = self.batch, self.S * self.S, self.device
        D = self.net.fc1_w.shape[1]
        self.D = D
        self.z = torch.zeros(B, NP, device=dev)
        self.h = torch.zeros(B, D, device=dev)
        self.dh = torch.zeros(B, D, device=dev)
        self.dzl = torch.zeros(B, NP, device=dev)
        self.val = torch.zeros(B, device=dev)
        self.dout = torch.zeros(B, D + 1, device=dev)
        self.dhead = torch.zeros(B, self.F + 1, device=dev)
        self.tval = torch.zeros(B, device=dev)

    def _forward_for_head(self, planes, targets, sym):
        self.forward_trunk(planes, sym, None, None)

    def _head_forward(self):
        v = self.fp.views
        ops.head_logits(self.Y[-1], v["head_w"].view(-1), v["head_b"], self.z, self.S)
        ops.dense_f32(self.z, v["fc1_w"], self.h, bias=v["fc1_b"])  # h = z W1 + b1

    def _head_train(self, targets, gscale, weight):
        v, gv = self.fp.views, self.fp.grad_views
        self._head_forward()
        self.tval.copy_(targets)
        ops.value_out(self.h, v["fc2_w"].view(-1), v["fc2_b"], self.val, target=self.tval, weight=weight,
                      loss=self.loss, correct=self.correct, dh=self.dh, dout=self.dout, grad_scale=gscale)
        ops.dense_f32(self.z, self.dh, gv["fc1_w"], trans_a=True)  # dW1 = z^T dh
        # column sums of the per-board partials on the fixed-order head_grad_sums kernel (torch's
        # column reductions were 4 launches, ~50 us of the 4.3 ms fp8 step); every call also writes
        # the step's (loss, correct) sums into a fresh 2-vector
        self._metric_sums = torch.empty(2, device=self.device)
        ops.head_grad_sums(self.dh, self.loss, self.correct, gv["fc1_b"], self._metric_sums)
        o2, n2 = self.fp.segments["fc2_w"]
        ops.head_grad_sums(self.dout, self.loss, self.correct, self.fp.grad[o2:o2 + n2 + 1],
                           self._metric_sums)  # [dw2 | db2]
        ops.dense_f32(self.dh, v["fc1_w"], self.dzl, trans_b=True)  # dz = dh W1^T
        # fp8 backward: dZ goes out as e5m2 straight from the head (no bf16 dZ write + quantize_bf8
        # re-read: 37 us of the 4.2 ms fp8 step, round 6)
        top = self.L - 1
        self._head_wrote_e5m2 = self._top_e5m2_fusable()
        e5 = (self.DZ8[top], self.gosc8[top:top + 1], self.gamax8[top]) if self._head_wrote_e5m2 else ()
        ops.head_backward(self.Y[-1], v["head_w"].view(-1), self.dzl, self.DZ[-1], self.dhead, self.S, *e5)
        ho, hn = self.fp.segments["head_w"]
        ops.head_grad_sums(self.dhead, self.loss, self.correct, self.fp.grad[ho:ho + hn + 1],
                           self._metric_sums)  # [dW_head | db_head]

    def _step_metrics(self):
        return self._metric_sums[0], self._metric_sums[1]

    @torch.no_grad()
    def evaluate(self, planes: torch.Tensor, targets: torch.Tensor):
        val = self.predict(planes)
        z = targets.float()
        return ((val - z) ** 2).sum(), (torch.sign(val) == torch.sign(z)).float().sum()

    @torch.no_grad()
    def predict(self, planes: torch.Tensor) -> torch.Tensor:
        self.forward_trunk(planes, None, None, None)
        self._head_forward()
        v = self.fp.views
        ops.value_out(self.h, v["fc2_w"].view(-1), v["fc2_b"], self.val)
        return self.val.clone()


class _TorchTrainerBase:
    def _setup(self, net, batch, lr, decay, device, dtype, iterations, named, optimizer="sgd", momentum=0.0,
               nesterov=False):
        self.env = agdist.env()
        self.device = torch.device(device) if device is not None else self.env.device
        self.net = net.to(self.device)
        self.batch = batch
        self.dtype = dtype
        self.sched = KerasSGDSchedule(lr, decay, iterations, optimizer=optimizer, momentum=momentum,
                                      nesterov=nesterov)
        self.params = [p for _, p in named]
        self.fp = FlatParams(named, self.device)
        if self.env.distributed:
            agdist.broadcast_(self.fp.flat, 0)
        self.opt_state = [torch.zeros_like(self.fp.flat) for _ in range(self.sched.n_moments)]
        self.table = symmetry_tables(net.board, self.device)

    def compute_grads(self, planes, targets, sym=None, weight=None, reduce: bool = True, rows=None):
        if rows is not None:  # the HIP trainers gather inside the pack kernel
            planes = planes.index_select(0, rows)
        for p in self.params:
            p.grad = None
        obj, per, metric = self._loss(planes, targets, sym, weight)
        obj.backward()
        for (name, p) in zip(self.fp.names, self.params):
            if p.grad is None:
                self.fp.grad_views[name].zero_()
            else:
                self.fp.grad_views[name].copy_(p.grad)
        if reduce and self.env.distributed:
            agdist.all_reduce_sum_(self.fp.grad)
        self._last = (per.detach(), metric.detach())

    def apply_update(self):
        with torch.no_grad():
            if self.sched.optimizer == "sgd":
                self.fp.flat.add_(self.fp.grad, alpha=-self.sched.current())
            else:
                optimizer_update_(self.fp.flat, self.fp.grad, self.opt_state, self.sched, self.sched.current())
        self.sched.advance()

    def step(self, planes, targets, sym=None, weight=None, rows=None):
        self.compute_grads(planes, targets, sym, weight, rows=rows)
        self.apply_update()
        per, metric = self._last
        return per.sum(), metric.sum()

    @torch.no_grad()
    def evaluate(self, planes, targets):
        obj, per, metric = self._loss(planes, targets, None, None)
        return per.sum(), metric.sum()


class TorchPolicyTrainer(_TorchTrainerBase):
    """Autograd implementation of the same SL/RL step (fp32 by default)."""

    policy_loss = "ce"  # or "bce" (reference RL loss), as HipPolicyTrainer

    def __init__(self, net: PolicyNet, batch: int, lr: float = 0.003, decay: float = 0.0, device=None,
                 dtype=torch.float32, iterations: int = 0, optimizer: str = "sgd", momentum: float = 0.0,
                 nesterov: bool = False):
        named = []
        tr = net.trunk
        for l in range(tr.layers):
            named.append(("w%d" % l, tr.weights[l]))
            named.append(("b%d" % l, tr.biases[l]))
        named += [("head_w", net.head_w), ("head_b", net.head_b)]
        self._setup(net, batch, lr, decay, device, dtype, iterations, named, optimizer, momentum, nesterov)

    def _loss(self, planes, targets, sym, weight):
        if sym is not None:
            planes, targets = apply_symmetry(planes, targets, sym, self.table)
        x = planes.to(self.dtype)
        logits = self.net.logits_torch(x)
        t = targets.long()
        valid = t >= 0
        correct = ((logits.argmax(1) == t) & valid).float()
        w = valid.float() if weight is None else valid.float() * weight
        norm = planes.shape[0] * self.env.world_size
        if self.policy_loss == "bce":
            # reference RL loss: Keras binary_crossentropy on the softmax output,
            # mean over the S*S outputs, clipped probabilities
            prob = torch.softmax(logits, 1).clamp(1e-7, 1 - 1e-7)
            y = torch.nn.functional.one_hot(t.clamp_min(0), logits.shape[1]).to(prob.dtype)
            per = -(y * prob.log() + (1 - y) * (1 - prob).log()).mean(1) * valid
            return (per * w).sum() / norm, per, correct
        logp = torch.log_softmax(logits, 1)
        lt = logp.gather(1, t.clamp_min(0).unsqueeze(1)).squeeze(1)
        per = -torch.clamp(lt, min=math.log(1e-7), max=math.log(1 - 1e-7)) * valid
        # gradient of mean CE (unclipped, see kernels/head.hip); optional per-board weights (REINFORCE)
        obj = (-(lt * w)).sum() / norm
        return obj, per, correct


class TorchValueTrainer(_TorchTrainerBase):
    def __init__(self, net: ValueNet, batch: int, lr: float = 0.003, decay: float = 0.0, device=None,
                 dtype=torch.float32, iterations: int = 0, optimizer: str = "sgd", momentum: float = 0.0,
                 nesterov: bool = False):
        named = []
        tr = net.trunk
        for l in range(tr.layers):
            named.append(("w%d" % l, tr.weights[l]))
            named.append(("b%d" % l, tr.biases[l]))
        named += [("head_w", net.head_w), ("head_b", net.head_b), ("fc1_w", net.fc1_w), ("fc1_b", net.fc1_b),
                  ("fc2_w", net.fc2_w), ("fc2_b", net.fc2_b)]
        self._setup(net, batch, lr, decay, device, dtype, iterations, named, optimizer, momentum, nesterov)

    def _loss(self, planes, targets, sym, weight):
        if sym is not None:
            planes, _ = apply_symmetry(planes, None, sym, self.table)
        v = self.net.forward_torch(planes.to(self.dtype))
        z = targets.float()
        err = (v - z) ** 2
        w = err if weight is None else err * weight
        obj = w.sum() / (planes.shape[0] * self.env.world_size)
        return obj, err, (torch.sign(v) == torch.sign(z)).float()


def make_value_trainer(net: ValueNet, batch: int, lr: float, decay: float = 0.0, backend: str = "auto",
                       device=None, **kw):
    dev = torch.device(device) if device is not None else agdist.env().device
    if backend == "auto":
        backend = "hip" if dev.type == "cuda" else "torch"
    if backend == "hip":
        return HipValueTrainer(net, batch, lr, decay, device=dev, **kw)
    return TorchValueTrainer(net, batch, lr, decay, device=dev, **_torch_kw(kw))


def make_policy_trainer(net: PolicyNet, batch: int, lr: float, decay: float = 0.0, backend: str = "auto",
                        device=None, **kw):
    dev = torch.device(device) if device is not None else agdist.env().device
    if backend == "auto":
        backend = "hip" if dev.type == "cuda" else "torch"
    if backend == "hip":
        return HipPolicyTrainer(net, batch, lr, decay, device=dev, **kw)
    return TorchPolicyTrainer(net, batch, lr, decay, device=dev, **_torch_kw(kw))


def _torch_kw(kw: dict) -> dict:
    """The HIP-trainer keywords the autograd trainers share (the rest are kernel options)."""
    return {k: kw[k] for k in ("iterations", "optimizer", "momentum", "nesterov") if k in kw}
