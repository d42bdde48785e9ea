"""Network definitions: policy CNN and value CNN.

Architecture parity with the reference Keras builders:

* policy (AlphaGo/models/policy.py:93-156): Conv(k1=5, F, ReLU, same) ->
  (layers-1) x Conv(k=3 or filter_width_K, F, ReLU, same) -> Conv(1x1, 1, linear,
  scalar bias) -> Flatten -> Softmax over S*S.  Defaults board=19, F=128,
  layers=12, Keras ``uniform`` init (U(-0.05, 0.05), zero bias).
* value (AlphaGo/models/value.py:12-31): 49 planes, Conv 5x5 K=152 ReLU,
  11 x Conv 3x3 ReLU, Conv 1x1 linear, Flatten, Dense(256, linear), Dense(1, tanh).

Parameters are kept as fp32 master tensors in PyTorch OIHW cross-correlation
layout.  Execution goes through one of two backends:

* ``"hip"`` — the MI355X path: hand-written CDNA4 kernels in
  ``alphago_amd.ops`` (implicit-GEMM conv on MFMA over zero-padded NHWC bf16,
  fused bias+ReLU epilogues, fused head/softmax/CE).
* ``"torch"`` — plain ``torch.nn.functional`` (the fp32 numerics oracle; also
  the CPU path).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

KERAS_UNIFORM_SCALE = 0.05


def keras_uniform_(t: torch.Tensor, scale: float = KERAS_UNIFORM_SCALE, generator=None) -> torch.Tensor:
    with torch.no_grad():
        return t.uniform_(-scale, scale, generator=generator)


def he_uniform_(net: nn.Module, generator=None) -> nn.Module:
    """Fan-in scaled uniform init (He for the ReLU trunk and the 1x1 head conv, LeCun for the dense
    layers) of a PolicyNet / ValueNet, biases zero: the reference's ``uniform(-0.05, 0.05)`` shrinks a
    12-layer trunk's signal ~30x (value.py:17,21), which plain SGD does not recover from."""
    with torch.no_grad():
        for w in list(net.trunk.weights) + [net.head_w]:
            bound = (6.0 / (w.shape[1] * w.shape[2] * w.shape[3])) ** 0.5
            w.uniform_(-bound, bound, generator=generator)
        for name in ("fc1_w", "fc2_w"):  # Keras (in, out) layout: fan_in = rows
            w = getattr(net, name, None)
            if w is not None:
                bound = (3.0 / w.shape[0]) ** 0.5
                w.uniform_(-bound, bound, generator=generator)
    return net


class ConvStack(nn.Module):
    """Shared trunk: conv(k_1) + (L-1) conv(k_i), all ReLU, 'same' padding."""

    def __init__(self, in_planes: int, filters: int, layers: int, widths: List[int]):
        super().__init__()
        assert len(widths) == layers
        for w in widths:
            if w % 2 != 1:
                raise ValueError("filter widths must be odd")
        self.in_planes, self.filters, self.layers, self.widths = in_planes, filters, layers, list(widths)
        self.weights = nn.ParameterList()
        self.biases = nn.ParameterList()
        cin = in_planes
        for w in widths:
            self.weights.append(nn.Parameter(torch.empty(filters, cin, w, w)))
            self.biases.append(nn.Parameter(torch.zeros(filters)))
            cin = filters
        self.reset_parameters()

    def reset_parameters(self, generator=None):
        for w in self.weights:
            keras_uniform_(w, generator=generator)
        for b in self.biases:
            nn.init.zeros_(b)

    def forward_torch(self, x: torch.Tensor) -> torch.Tensor:
        for w, b, k in zip(self.weights, self.biases, self.widths):
            x = F.relu(F.conv2d(x, w.to(x.dtype), b.to(x.dtype), padding=k // 2))
        return x


class PolicyNet(nn.Module):
    """SL/RL policy network (reference CNNPolicy.create_network)."""

    def __init__(self, input_dim: int, board: int = 19, filters_per_layer: int = 128, layers: int = 12,
                 **kwargs):
        super().__init__()
        widths = [int(kwargs.get("filter_width_%d" % i, 5 if i == 1 else 3)) for i in range(1, layers + 1)]
        self.arch = dict(input_dim=input_dim, board=board, filters_per_layer=filters_per_layer, layers=layers)
        for i, w in enumerate(widths, 1):
            if (i == 1 and w != 5) or (i > 1 and w != 3):
                self.arch["filter_width_%d" % i] = w
        self.board = board
        self.trunk = ConvStack(input_dim, filters_per_layer, layers, widths)
        self.head_w = nn.Parameter(torch.empty(1, filters_per_layer, 1, 1))
        self.head_b = nn.Parameter(torch.zeros(1))
        keras_uniform_(self.head_w)

    @property
    def input_dim(self):
        return self.arch["input_dim"]

    def logits_torch(self, x: torch.Tensor) -> torch.Tensor:
        h = self.trunk.forward_torch(x)
        z = F.conv2d(h, self.head_w.to(h.dtype), self.head_b.to(h.dtype))
        return z.flatten(1).float()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: (B, C, S, S) float/uint8 planes -> (B, S*S) move probabilities."""
        if x.dtype == torch.uint8:
            x = x.float()
        return torch.softmax(self.logits_torch(x), dim=1)

    def flops_per_position(self) -> float:
        """Forward FLOPs per board (2*MACs), exact for stride-1 'same' convs."""
        s2 = self.board * self.board
        tot = 0.0
        cin = self.trunk.in_planes
        for k in self.trunk.widths:
            tot += 2.0 * s2 * cin * self.trunk.filters * k * k
            cin = self.trunk.filters
        tot += 2.0 * s2 * cin
        return tot


class ValueNet(nn.Module):
    """Value network (reference value.py:12-31) with a tanh scalar output."""

    def __init__(self, input_dim: int = 49, board: int = 19, filters_per_layer: int = 152, layers: int = 12,
                 dense: int = 256, **kwargs):
        super().__init__()
        widths = [int(kwargs.get("filter_width_%d" % i, 5 if i == 1 else 3)) for i in range(1, layers + 1)]
        self.arch = dict(input_dim=input_dim, board=board, filters_per_layer=filters_per_layer, layers=layers,
                         dense=dense)
        self.board = board
        self.trunk = ConvStack(input_dim, filters_per_layer, layers, widths)
        self.head_w = nn.Parameter(torch.empty(1, filters_per_layer, 1, 1))
        self.head_b = nn.Parameter(torch.zeros(1))
        self.fc1_w = nn.Parameter(torch.empty(board * board, dense))  # Keras Dense layout (in, out)
        self.fc1_b = nn.Parameter(torch.zeros(dense))
        self.fc2_w = nn.Parameter(torch.empty(dense, 1))
        self.fc2_b = nn.Parameter(torch.zeros(1))
        for p in (self.head_w, self.fc1_w, self.fc2_w):
            keras_uniform_(p)

    @property
    def input_dim(self):
        return self.arch["input_dim"]

    def flops_per_position(self) -> float:
        """Forward FLOPs per board (2*MACs): trunk, 1x1 head conv, Dense(S*S -> dense), Dense(dense -> 1)."""
        s2 = self.board * self.board
        tot, cin = 0.0, self.trunk.in_planes
        for k in self.trunk.widths:
            tot += 2.0 * s2 * cin * self.trunk.filters * k * k
            cin = self.trunk.filters
        d = self.arch["dense"]
        return tot + 2.0 * s2 * cin + 2.0 * s2 * d + 2.0 * d

    def forward_torch(self, x: torch.Tensor) -> torch.Tensor:
        h = self.trunk.forward_torch(x)
        z = F.conv2d(h, self.head_w.to(h.dtype), self.head_b.to(h.dtype)).flatten(1).float()
        z = z @ self.fc1_w + self.fc1_b  # linear (value.py:27)
        return torch.tanh(z @ self.fc2_w + self.fc2_b).squeeze(1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.dtype == torch.uint8:
            x = x.float()
        return self.forward_torch(x)
