"""Batched network evaluation for play, search and self-play.

On a GPU the whole forward (uint8 planes -> padded NHWC bf16 -> L x MFMA conv
-> fused head/softmax with legal-move renormalisation) is captured once per
batch bucket into a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm) and
replayed: a search step is one H2D copy, one graph launch and one D2H copy,
instead of ~15 kernel launches.  Batches are padded up to the next bucket.

With a feature list, ``evaluate_encoded`` takes the engine's compact board
encoding (~2 bytes/point, ``Forest.leaf_encode_into`` / ``encode_batch``)
instead of uint8 planes: the GPU featurizer (ops/gpu_features.py) runs as the
first node of the same graph, writing the conv input and the sensible-move
mask directly (24x less H2D traffic than 48 uint8 planes, no CPU featurizing).

Reference paths replaced: CNNPolicy.forward / batch_eval_state
(policy.py:26-79) which featurised in Python and ran a Theano function per
call; MCTS policy/value callables (mcts.py:107-118).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from .nets import PolicyNet, ValueNet

DEFAULT_BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024)


class _Bucket:
    pass


class HipTrunkInference:
    """Forward-only runner of a ConvStack (+ head) on the HIP kernels."""

    def __init__(self, net, device, buckets: Sequence[int] = DEFAULT_BUCKETS, use_graphs: bool = True,
                 feature_list: Optional[Sequence[str]] = None, precision: Optional[str] = None):
        ops.load()
        self.net = net
        self.precision = precision or os.environ.get("ALPHAGO_AMD_PRECISION", "bf16")
        if self.precision not in ("bf16", "fp8"):
            raise ValueError("precision must be bf16 or fp8")
        self.device = torch.device(device)
        tr = net.trunk
        self.S, self.L, self.K = net.board, tr.layers, list(tr.widths)
        self.C0, self.F = tr.in_planes, tr.filters
        self.C0p = ops.round_up(self.C0, 64)
        self.Fp = ops.pad_filters(self.F)
        self.P0 = self.K[0] // 2
        self.buckets = sorted(buckets)
        self.use_graphs = use_graphs
        # fp8 engines run buckets below this many boards on the bf16 trunk: the fp8 forward's 384-pixel
        # tiles leave a small batch with a handful of workgroups (~480 us per policy forward at B <= 64 vs
        # 185-325 us bf16; even at B = 128, 520 / 451 us vs 515 / 427 bf16 for policy / value; fp8 wins
        # from B = 256 on, 578 / 488 us vs 817 / 702; profiles/r4/README.md); ALPHAGO_AMD_FP8_MIN_BATCH
        # overrides
        self.fp8_min_batch = int(os.environ.get("ALPHAGO_AMD_FP8_MIN_BATCH", "256"))
        dev = self.device
        # packed on the engine's device whatever device the module's parameters are on
        self.wf = [ops.packed_weight_like(tr.weights[l], self.C0p if l == 0 else self.Fp, self.Fp, device=dev)
                   for l in range(self.L)]
        # weight-stationary copies (tile 40, small buckets) of the layers that kernel covers
        self.wf_ws = [ops.ws_packed_like(self.wf[l]) if ops.conv_ws_supported(self.Fp, self.C0p if l == 0 else self.Fp,
                                                                              self.K[l]) else None
                      for l in range(self.L)]
        self.bias_p = [torch.zeros(self.Fp, device=dev) for _ in range(self.L)]
        self.head_w = torch.zeros(self.F, device=dev)
        self.head_b = torch.zeros(1, device=dev)
        self._b: Dict[int, _Bucket] = {}
        if self.precision == "fp8":
            L = self.L
            self.w8: List[torch.Tensor] = [None] * L
            self.ew = [0] * L
            self.ex = [0] * (L + 1)  # e4m3 exponent of each layer's input (layer 0: binary planes, exact at 0)
            self.scales8 = torch.full((L, 2), 127, dtype=torch.int32, device=dev)
            self.osc8 = torch.ones(L, device=dev)
            self.amax8 = ops.fp8_amax_buffer(L, dev)
            self.calibrated = False
        # encoded path: also write the uint8 planes of every board into the bucket (RL learner records
        # stay on the device, search/selfplay.py); toggled before capture (set_encoded_planes)
        self.encoded_planes = False
        self._last_bk = None
        self.fz = None
        if feature_list is not None:
            from ..ops.gpu_features import GpuFeaturizer
            fz = GpuFeaturizer(feature_list, board=self.S, device=dev)
            if fz.nplanes != self.C0:
                raise ValueError("feature list has %d planes, network expects %d" % (fz.nplanes, self.C0))
            self.fz = fz
        self.sync_weights()

    @property
    def supports_encoded(self) -> bool:
        return self.fz is not None

    @property
    def needs_ladder(self) -> bool:
        """Whether callers must encode ladder bits on the host (False when the
        GPU featurizer reads ladders on the device)."""
        return self.fz is not None and self.fz.host_needs_ladder

    @torch.no_grad()
    def sync_weights(self) -> None:
        tr = self.net.trunk
        ws = [w.detach().to(self.device, torch.float32).contiguous() for w in tr.weights]
        ops.pack_weights(ws, self.wf)
        ops.ws_pack([self.wf[l] for l in range(self.L) if self.wf_ws[l] is not None],
                    [w for w in self.wf_ws if w is not None])
        for l in range(self.L):
            self.bias_p[l][:self.F].copy_(tr.biases[l].detach())
        self.head_w.copy_(self.net.head_w.detach().view(-1))
        self.head_b.copy_(self.net.head_b.detach().view(-1))
        if self.precision == "fp8":
            for l in range(self.L):
                self.w8[l], self.ew[l] = ops.pack_weights_fp8(ws[l], self.Fp, self.C0p if l == 0 else self.Fp)
                self.scales8[l, 1] = 127 - self.ew[l]
            self.calibrated = False  # activation ranges change with the weights
        self._after_sync()

    def _after_sync(self):
        pass

    def bucket_for(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        return ops.round_up(n, self.buckets[-1])

    def _make_bucket(self, B: int) -> _Bucket:
        dev, S = self.device, self.S
        bk = _Bucket()
        bk.B = B
        bk.planes = torch.zeros((B, self.C0, S, S), dtype=torch.uint8, device=dev)
        bk.legal = torch.ones((B, S * S), dtype=torch.uint8, device=dev)
        bk.X0 = ops.padded_empty(B, S, self.P0, self.C0p, dev)
        bk.Y = [ops.padded_empty(B, S, 1, self.Fp, dev) for _ in range(2)]
        # small buckets: the split-K 32-pixel conv (ops.conv_fwd_splitk), fp32 partials in bk.ws
        M = B * S * S
        bk.sk = [1 if (self.precision == "fp8" and B >= self.fp8_min_batch) else
                 ops.splitk_nsplit(M, self.Fp, self.C0p if l == 0 else self.Fp, self.K[l]) for l in range(self.L)]
        # ... or the weight-stationary kernel (tile 40) where it applies (it replaces split-K there)
        bk.wst = [self.precision != "fp8" or B < self.fp8_min_batch for _ in range(self.L)]
        bk.wst = [bk.wst[l] and self.wf_ws[l] is not None and
                  ops.ws_applies(M, self.Fp, self.C0p if l == 0 else self.Fp, self.K[l]) for l in range(self.L)]
        bk.sk = [1 if bk.wst[l] else bk.sk[l] for l in range(self.L)]
        bk.ws = torch.empty(max(bk.sk) * M * self.Fp, device=dev) if max(bk.sk) > 1 else None
        if self.precision == "fp8":
            bk.X08 = torch.zeros(bk.X0.shape, dtype=torch.uint8, device=dev)
            bk.Y8 = [torch.zeros(bk.Y[0].shape, dtype=torch.uint8, device=dev) for _ in range(2)]
        self._alloc_outputs(bk)
        bk.graph = None
        bk.graph_enc = None
        if self.fz is not None:
            NP = S * S
            bk.e_board = torch.zeros((B, NP), dtype=torch.int8, device=dev)
            bk.e_ages = torch.full((B, NP), 255, dtype=torch.uint8, device=dev)
            bk.e_meta = torch.tensor([[-1, 1]] * B, dtype=torch.int32, device=dev)
            bk.e_ladder = torch.zeros((B, NP), dtype=torch.uint8, device=dev) if self.fz.need_ladder else None
            bk.ovf = torch.zeros((B,), dtype=torch.int32, device=dev)
        return bk

    def _alloc_outputs(self, bk):
        bk.probs = torch.zeros((bk.B, self.S * self.S), device=self.device)

    def set_encoded_planes(self, on: bool) -> None:
        """Make the encoded path also write uint8 planes (``encoded_planes_view``); re-captures graphs."""
        if bool(on) != self.encoded_planes:
            self.encoded_planes = bool(on)
            for bk in self._b.values():
                bk.graph_enc = None

    def encoded_planes_view(self, n: int) -> torch.Tensor:
        """(n, C, S, S) uint8 device planes of the last encoded submission (valid until the bucket is
        submitted again); needs ``set_encoded_planes(True)``."""
        if not self.encoded_planes or self._last_bk is None:
            raise RuntimeError("encoded planes are off")
        return self._last_bk.planes[:n]

    def _trunk(self, bk, encoded: bool = False) -> torch.Tensor:
        if encoded:
            bk.ovf.zero_()
            self.fz.run(bk.e_board, bk.e_ages, bk.e_meta, bk.e_ladder, nhwc=bk.X0, P=self.P0, sensible=bk.legal,
                        overflow=bk.ovf, planes=bk.planes if self.encoded_planes else None)
        else:
            ops.pack_input(bk.planes, bk.X0, self.P0)
        if self.precision == "fp8" and not getattr(self, "_calibrating", False) and bk.B >= self.fp8_min_batch:
            return self._trunk_fp8(bk)
        x, pin = bk.X0, self.P0
        for l in range(self.L):
            y = bk.Y[l % 2]
            if bk.wst[l]:
                ops.conv_fwd(x, self.wf_ws[l], self.bias_p[l], y, self.K[l], self.S, pin, 1, tile=40)
            elif bk.sk[l] > 1:
                ops.conv_fwd_splitk(x, self.wf[l], self.bias_p[l], y, self.K[l], self.S, pin, 1, ops.MODE_BIAS_RELU,
                                    None, bk.ws, bk.sk[l])
            else:
                ops.conv_fwd(x, self.wf[l], self.bias_p[l], y, self.K[l], self.S, pin, 1)
            if getattr(self, "_calibrating", False):
                self._cal_amax[l] = max(self._cal_amax[l], float(y.amax()))
            x, pin = y, 1
        return x

    # ------------------------------------------------------------------ fp8
    def _trunk_fp8(self, bk) -> torch.Tensor:
        """e4m3 trunk on the block-scaled MFMA: every layer reads and (but the
        last) writes e4m3 activations; the last writes bf16 for the head."""
        ops.quantize_fp8(bk.X0, bk.X08, 0)  # 0/1 planes are exact in e4m3
        x8, pin = bk.X08, self.P0
        for l in range(self.L):
            last = l == self.L - 1
            ops.conv_fwd_fp8(x8, self.w8[l], self.bias_p[l], self.scales8[l], self.osc8[l:l + 1], self.K[l], self.S,
                             pin, 1, y_bf16=bk.Y[0] if last else None, y_fp8=None if last else bk.Y8[l % 2],
                             amax=self.amax8[l])
            x8, pin = bk.Y8[l % 2], 1
        return bk.Y[0]

    @torch.no_grad()
    def calibrate(self, bk, encoded: bool = False, margin: int = 1) -> None:
        """Set per-layer e4m3 activation scales from a bf16 forward of the
        current bucket inputs (delayed scaling afterwards: recalibrate())."""
        self._cal_amax = [0.0] * self.L
        self._calibrating = True
        try:
            self._trunk(bk, encoded)
        finally:
            self._calibrating = False
        self._set_act_exponents([ops.fp8_exponent(a, margin) for a in self._cal_amax])
        self.calibrated = True

    def recalibrate(self, margin: int = 1) -> None:
        """Re-derive activation scales from the running amax tracked by the fp8 kernels."""
        amax = self.amax8.view(torch.float32).amax(1).tolist()
        self._set_act_exponents([ops.fp8_exponent(a, margin) for a in amax])

    def _set_act_exponents(self, out_exp) -> None:
        self.ex = [0] + list(out_exp)
        for l in range(self.L):
            self.scales8[l, 0] = 127 - self.ex[l]
            self.osc8[l] = 2.0 ** self.ex[l + 1]

    def _head(self, bk, y):
        ops.policy_head_probs(y, self.head_w, self.head_b, bk.probs, self.S, legal=bk.legal)

    def _run(self, bk, encoded: bool = False):
        self._head(bk, self._trunk(bk, encoded))

    def _capture(self, bk, encoded: bool):
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._run(bk, encoded)  # warm-up (also sets kernel attributes outside capture)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._run(bk, encoded)
        return g

    def _get(self, n: int, encoded: bool = False, slot: int = 0) -> _Bucket:
        B = self.bucket_for(n)
        key = (B, slot)
        if key not in self._b:
            self._b[key] = self._make_bucket(B)
        bk = self._b[key]
        if self.use_graphs:
            if encoded and bk.graph_enc is None:
                bk.graph_enc = self._capture(bk, True)
            elif not encoded and bk.graph is None:
                bk.graph = self._capture(bk, False)
        return bk

    @torch.no_grad()
    def submit_encoded(self, board, ages, meta, ladder=None, slot: int = 0, to_host: bool = False):
        """Asynchronous half of evaluate_encoded: H2D copies (non-blocking from
        pinned host buffers) + graph replay on the current stream; with
        ``to_host`` also the D2H copy of the results into pinned host buffers,
        followed by an event.  ``slot`` selects an independent set of bucket
        buffers, so two batches can be in flight; the GPU work stays serial on
        one stream (two overlapping batches would delay each other's results).
        Returns a handle for collect()."""
        assert self.fz is not None, "engine built without a feature list"
        n = board.shape[0]
        bk = self._get(n, encoded=True, slot=slot)
        bk.e_board[:n].copy_(torch.as_tensor(board), non_blocking=True)
        bk.e_ages[:n].copy_(torch.as_tensor(ages), non_blocking=True)
        bk.e_meta[:n].copy_(torch.as_tensor(meta), non_blocking=True)
        if bk.e_ladder is not None and self.fz.host_needs_ladder:
            if ladder is None:
                raise ValueError("this feature list needs ladder bits")
            bk.e_ladder[:n].copy_(torch.as_tensor(ladder), non_blocking=True)
        if n < bk.B:
            bk.e_board[n:].zero_()
            bk.e_ages[n:].fill_(255)
        if self.precision == "fp8" and not self.calibrated:
            self.calibrate(bk, encoded=True)
        if bk.graph_enc is not None:
            bk.graph_enc.replay()
        else:
            self._run(bk, True)
        self._last_bk = bk
        host = None
        if to_host:
            if not hasattr(bk, "h_out"):
                out = self._outputs(bk, bk.B)
                bk.h_out = torch.empty(out.shape, dtype=torch.float32, pin_memory=True)
                bk.h_mask = torch.empty(bk.legal.shape, dtype=torch.uint8, pin_memory=True)
                bk.h_ovf = torch.empty(bk.ovf.shape, dtype=torch.int32, pin_memory=True)
            bk.h_out[:n].copy_(self._outputs(bk, n), non_blocking=True)
            bk.h_mask[:n].copy_(bk.legal[:n], non_blocking=True)
            bk.h_ovf[:n].copy_(bk.ovf[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            host = ev
        return bk, n, host

    def collect(self, handle):
        """(outputs (n, ...), sensible mask (n, S*S), overflow board indices).
        For a to_host submission: numpy views of the pinned host buffers (valid
        until the slot is submitted again), waiting only for that batch's event."""
        bk, n, ev = handle
        if ev is not None:
            ev.synchronize()
            bad = np.nonzero(bk.h_ovf[:n].numpy())[0].tolist()
            return bk.h_out[:n].numpy(), bk.h_mask[:n].numpy(), bad
        bad = torch.nonzero(bk.ovf[:n]).flatten().tolist()
        return self._outputs(bk, n), bk.legal[:n], bad

    def outputs(self, handle):
        """Device views (outputs (n, ...), sensible mask (n, S*S) uint8) of a submission, no waiting."""
        bk, n, _ = handle
        return self._outputs(bk, n), bk.legal[:n]

    @torch.no_grad()
    def evaluate_encoded(self, board, ages, meta, ladder=None, slot: int = 0):
        """Forward from the compact encoding (GPU featurizer in the graph).

        Returns (outputs (n, ...), sensible mask (n, S*S) uint8 device tensor,
        list of board indices whose eye recursion overflowed the kernel and
        must be re-evaluated from CPU planes)."""
        return self.collect(self.submit_encoded(board, ages, meta, ladder, slot))

    @torch.no_grad()
    def evaluate(self, planes, legal=None, slot: int = 0):
        """planes: (n, C, S, S) uint8 (numpy or tensor); legal: (n, S*S) uint8 or None.
        Returns the bucket's output tensors (views of the first n rows).  ``slot`` selects the
        bucket buffers as in submit_encoded (a caller with encoded batches in flight uses a slot
        none of them holds)."""
        n = planes.shape[0]
        bk = self._get(n, encoded=False, slot=slot)
        src = torch.as_tensor(planes)
        bk.planes[:n].copy_(src, non_blocking=True)
        if n < bk.B:
            bk.planes[n:].zero_()
        if legal is not None:
            bk.legal[:n].copy_(torch.as_tensor(legal), non_blocking=True)
            if n < bk.B:
                bk.legal[n:].fill_(1)
        else:
            bk.legal.fill_(1)
        if self.precision == "fp8" and not self.calibrated:
            self.calibrate(bk)
        if bk.graph is not None:
            bk.graph.replay()
        else:
            self._run(bk)
        return self._outputs(bk, n)

    def _outputs(self, bk, n):
        return bk.probs[:n]


class HipValueInference(HipTrunkInference):
    """Value net: HIP trunk, then the head as head_logits (1x1 conv) -> dense_f32
    (Dense 256, fp32 MFMA GEMM) -> value_out (Dense 1 + tanh), all inside the
    captured graph."""

    def __init__(self, net: ValueNet, device, **kw):
        self.fc = None
        super().__init__(net, device, **kw)

    def _after_sync(self):
        n = self.net
        self.fc = [t.detach().to(self.device, torch.float32).clone() for t in (n.fc1_w, n.fc1_b, n.fc2_w, n.fc2_b)]

    def _alloc_outputs(self, bk):
        bk.values = torch.zeros((bk.B,), device=self.device)
        bk.z = torch.zeros((bk.B, self.S * self.S), device=self.device)
        bk.h = torch.zeros((bk.B, self.fc[0].shape[1]), device=self.device)

    def _head(self, bk, y):
        w1, b1, w2, b2 = self.fc
        ops.head_logits(y, self.head_w, self.head_b, bk.z, self.S)
        ops.dense_f32(bk.z, w1, bk.h, bias=b1)
        ops.value_out(bk.h, w2.view(-1), b2, bk.values)

    def _outputs(self, bk, n):
        return bk.values[:n]


class TorchPolicyInference:
    """CPU / reference path with the same interface."""

    supports_encoded = False
    needs_ladder = False

    def __init__(self, net: PolicyNet, device="cpu"):
        self.net, self.device = net, torch.device(device)

    def sync_weights(self):
        pass

    @torch.no_grad()
    def evaluate(self, planes, legal=None, slot: int = 0):
        x = torch.as_tensor(planes).to(self.device)
        logits = self.net.logits_torch(x.float())
        if legal is not None:
            logits = logits.masked_fill(torch.as_tensor(legal).to(self.device) == 0, float("-inf"))
        p = torch.softmax(logits, 1)
        return torch.nan_to_num(p, nan=0.0)


class TorchValueInference:
    supports_encoded = False
    needs_ladder = False

    def __init__(self, net: ValueNet, device="cpu"):
        self.net, self.device = net, torch.device(device)

    def sync_weights(self):
        pass

    @torch.no_grad()
    def evaluate(self, planes, legal=None, slot: int = 0):
        return self.net.forward_torch(torch.as_tensor(planes).to(self.device).float())


def make_policy_inference(net, device, **kw):
    """HIP engine on a GPU (pass ``feature_list`` to enable evaluate_encoded), torch on CPU."""
    device = torch.device(device)
    if device.type == "cuda":
        return HipTrunkInference(net, device, **kw)
    return TorchPolicyInference(net, device)  # feature_list unused: CPU featurizer path


def make_value_inference(net, device, **kw):
    device = torch.device(device)
    if device.type == "cuda":
        return HipValueInference(net, device, **kw)
    return TorchValueInference(net, device)  # feature_list unused: CPU featurizer path
