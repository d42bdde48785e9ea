"""Keras-1.0-compatible model files.

Model JSON (reference CNNPolicy.save_model, policy.py:171-193):
    {"keras_model": "<Keras 1.0 Sequential JSON>", "feature_list": [...],
     "weights_file": "<path>"?}
Weights HDF5 (Keras 1.0 ``save_weights``): root attribute ``layer_names``; one
group per layer with attribute ``weight_names`` and datasets ``<layer>_W`` /
``<layer>_b``.  Conv kernels are (nb_filter, stack, rows, cols); Dense kernels
(input_dim, output_dim).  Weights load *by layer order* like Keras does.

Kernel orientation: Keras-on-Theano uses Theano's true convolution (flipped
kernels), our kernels are cross-correlations, so conv kernels are flipped on
save/load by default (``kernel_flip=True``).  Pass
``kernel_flip=False`` for files written by a cross-correlation backend.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..models.nets import PolicyNet, ValueNet
from .h5lite import H5File, H5Writer

_NULLS = {"W_constraint": None, "W_regularizer": None, "activity_regularizer": None, "b_constraint": None,
          "b_regularizer": None}


def _conv_cfg(name, nb_filter, k, activation, input_shape=None):
    cfg = dict(_NULLS)
    cfg.update({"activation": activation, "border_mode": "same", "dim_ordering": "th", "init": "uniform",
                "name": name, "nb_col": k, "nb_filter": nb_filter, "nb_row": k, "subsample": [1, 1],
                "trainable": True})
    if input_shape is not None:
        cfg["batch_input_shape"] = [None] + list(input_shape)
        cfg["input_dtype"] = "float32"
    return {"class_name": "Convolution2D", "config": cfg}


def _dense_cfg(name, output_dim, activation):
    cfg = dict(_NULLS)
    cfg.update({"activation": activation, "bias": True, "init": "uniform", "input_dim": None, "name": name,
                "output_dim": output_dim, "trainable": True})
    return {"class_name": "Dense", "config": cfg}


def _layer_names(net) -> List[str]:
    n = net.trunk.layers + 1
    names = ["convolution2d_%d" % (i + 1) for i in range(n)] + ["flatten_1"]
    if isinstance(net, ValueNet):
        names += ["dense_1", "dense_2"]
    else:
        names += ["activation_1"]
    return names


def model_to_keras_json(net) -> str:
    tr = net.trunk
    names = _layer_names(net)
    layers = []
    for i, k in enumerate(tr.widths):
        layers.append(_conv_cfg(names[i], tr.filters, k, "relu",
                                (tr.in_planes, net.board, net.board) if i == 0 else None))
    layers.append(_conv_cfg(names[tr.layers], 1, 1, "linear"))
    layers.append({"class_name": "Flatten", "config": {"name": "flatten_1", "trainable": True}})
    if isinstance(net, ValueNet):
        layers.append(_dense_cfg("dense_1", net.arch["dense"], "linear"))
        layers.append(_dense_cfg("dense_2", 1, "tanh"))
    else:
        layers.append({"class_name": "Activation", "config": {"activation": "softmax", "name": "activation_1",
                                                               "trainable": True}})
    return json.dumps({"class_name": "Sequential", "config": layers})


def model_from_keras_json(spec: str):
    """Build a PolicyNet or ValueNet from a Keras 1.0 Sequential JSON string."""
    d = json.loads(spec) if isinstance(spec, str) else spec
    if d.get("class_name") != "Sequential":
        raise ValueError("only Sequential models are supported")
    cfgs = d["config"]
    if isinstance(cfgs, dict):  # Keras >= 1.2 wraps layers
        cfgs = cfgs.get("layers", cfgs)
    convs = [c["config"] for c in cfgs if c["class_name"] == "Convolution2D"]
    denses = [c["config"] for c in cfgs if c["class_name"] == "Dense"]
    if len(convs) < 2:
        raise ValueError("expected >= 2 convolution layers")
    first = convs[0]
    shape = first.get("batch_input_shape") or [None] + list(first.get("input_shape", []))
    input_dim, board = int(shape[1]), int(shape[2])
    trunk = convs[:-1]
    filters = int(trunk[0]["nb_filter"])
    kw = {}
    for i, c in enumerate(trunk, 1):
        kw["filter_width_%d" % i] = int(c["nb_row"])
    if denses:
        return ValueNet(input_dim=input_dim, board=board, filters_per_layer=filters, layers=len(trunk),
                        dense=int(denses[0]["output_dim"]), **kw)
    return PolicyNet(input_dim, board=board, filters_per_layer=filters, layers=len(trunk), **kw)


def _weights_in_order(net) -> List[Tuple[str, List[torch.Tensor]]]:
    names = _layer_names(net)
    tr = net.trunk
    out = []
    for i in range(tr.layers):
        out.append((names[i], [tr.weights[i], tr.biases[i]]))
    out.append((names[tr.layers], [net.head_w, net.head_b]))
    out.append(("flatten_1", []))
    if isinstance(net, ValueNet):
        out.append(("dense_1", [net.fc1_w, net.fc1_b]))
        out.append(("dense_2", [net.fc2_w, net.fc2_b]))
    else:
        out.append(("activation_1", []))
    return out


def save_weights(net, path: str, kernel_flip: bool = True) -> None:
    layers = _weights_in_order(net)
    with H5Writer(path) as f:
        f.attrs["layer_names"] = np.array([n.encode() for n, _ in layers])
        for name, ws in layers:
            g = f.create_group(name)
            wn = [name + "_W", name + "_b"] if ws else []
            g.attrs["weight_names"] = np.array([w.encode() for w in wn]) if wn else np.zeros((0,), "S1")
            for wname, t in zip(wn, ws):
                a = t.detach().float().cpu().numpy()
                if wname.endswith("_W") and a.ndim == 4 and kernel_flip:
                    a = a[:, :, ::-1, ::-1]
                g[wname] = np.array(a, dtype=np.float32, order="C", copy=True)


def load_weights(net, path: str, kernel_flip: bool = True) -> None:
    layers = [ws for _, ws in _weights_in_order(net) if ws]
    with H5File(path) as f:
        names = [n.decode() if isinstance(n, bytes) else str(n) for n in f.attrs["layer_names"]]
        groups = []
        for n in names:
            g = f[n]
            wn = g.attrs.get("weight_names", [])
            wn = [w.decode() if isinstance(w, bytes) else str(w) for w in np.atleast_1d(wn)]
            if wn:
                groups.append([g[w].read() for w in wn])
        if len(groups) != len(layers):
            raise ValueError("weight file has %d weighted layers, model has %d" % (len(groups), len(layers)))
        with torch.no_grad():
            for arrs, params in zip(groups, layers):
                for a, p in zip(arrs, params):
                    a = np.asarray(a, dtype=np.float32)
                    if a.ndim == 4 and kernel_flip:
                        a = a[:, :, ::-1, ::-1]
                    a = a.reshape(tuple(p.shape)) if a.size == p.numel() else a
                    if tuple(a.shape) != tuple(p.shape):
                        raise ValueError("shape mismatch %s vs %s" % (a.shape, tuple(p.shape)))
                    p.data.copy_(torch.from_numpy(np.array(a, dtype=np.float32, order="C", copy=True)))
