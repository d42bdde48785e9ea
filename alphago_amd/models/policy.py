"""CNNPolicy / CNNValue: reference-compatible model wrappers.

API parity with the reference CNNPolicy (AlphaGo/models/policy.py:12-193):
``CNNPolicy(feature_list, **arch)``, ``.forward``, ``.eval_state``,
``.batch_eval_state``, ``create_network``, ``load_model``, ``save_model``,
``.model``, ``.preprocessor``.  The network is a torch module; evaluation runs
through :mod:`alphago_amd.models.inference` (HIP graphs on the GPU, torch on
CPU).  Featurisation is native C++ (batched, multithreaded).
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..features import DEFAULT_FEATURES, VALUE_FEATURES, Preprocess
from ..io import keras_compat
from ..utils.gorecords import flatten_idx
from .inference import make_policy_inference, make_value_inference
from .nets import PolicyNet, ValueNet


def default_device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class _NetWrapper(object):
    _net_cls = PolicyNet

    def __init__(self, feature_list: Sequence[str], device=None, **kwargs):
        self.preprocessor = Preprocess(feature_list)
        kwargs["input_dim"] = self.preprocessor.output_dim
        self.device = torch.device(device) if device is not None else default_device()
        self.model = self.create_network(**kwargs).to(self.device)
        self._engine = None

    @classmethod
    def create_network(cls, **kwargs):
        return cls._net_cls(**kwargs)

    def _engine_kw(self):
        """GPU engines get the feature list so they can featurize on the device."""
        if self.device.type == "cuda" and self.preprocessor.output_dim <= 64:
            return {"feature_list": self.preprocessor.feature_list}
        return {}

    @property
    def engine(self):
        if self._engine is None:
            self._engine = self._make_engine()
        return self._engine

    def refresh(self) -> None:
        """Re-read weights into the inference engine after training updates."""
        if self._engine is not None:
            self._engine.sync_weights()

    # ---------------------------------------------------------- persistence
    def save_model(self, json_file: str, weights_file: Optional[str] = None) -> None:
        specs = {"keras_model": keras_compat.model_to_keras_json(self.model),
                 "feature_list": self.preprocessor.feature_list}
        if weights_file is not None:
            keras_compat.save_weights(self.model, weights_file)
            specs["weights_file"] = weights_file
        with open(json_file, "w") as f:
            json.dump(specs, f)

    @classmethod
    def load_model(cls, json_file: str, device=None, weights_file: Optional[str] = None):
        with open(json_file, "r") as f:
            specs = json.load(f)
        obj = cls.__new__(cls)
        obj.preprocessor = Preprocess(specs["feature_list"])
        obj.device = torch.device(device) if device is not None else default_device()
        net = keras_compat.model_from_keras_json(specs["keras_model"])
        if not isinstance(net, cls._net_cls):
            raise ValueError("%s expects a %s spec" % (cls.__name__, cls._net_cls.__name__))
        obj.model = net.to(obj.device)
        obj._engine = None
        wf = weights_file or specs.get("weights_file")
        if wf:
            if not os.path.isabs(wf) and not os.path.exists(wf):
                wf = os.path.join(os.path.dirname(os.path.abspath(json_file)), wf)
            keras_compat.load_weights(obj.model, wf)
        return obj

    def load_weights(self, weights_file: str) -> None:
        keras_compat.load_weights(self.model, weights_file)
        self.refresh()

    def save_weights(self, weights_file: str) -> None:
        keras_compat.save_weights(self.model, weights_file)


class CNNPolicy(_NetWrapper):
    """Policy network: state -> distribution over moves."""

    _net_cls = PolicyNet

    def __init__(self, feature_list: Sequence[str] = DEFAULT_FEATURES, device=None, **kwargs):
        super().__init__(feature_list, device=device, **kwargs)

    def _make_engine(self):
        return make_policy_inference(self.model, self.device, **self._engine_kw())

    def forward(self, planes, legal=None) -> np.ndarray:
        """(B, F, S, S) planes -> (B, S*S) probabilities (numpy)."""
        planes = np.asarray(planes)
        if planes.dtype != np.uint8:
            planes = planes.astype(np.uint8)
        return self.engine.evaluate(planes, legal).float().cpu().numpy()

    def batch_eval_state(self, states, moves_lists=None):
        """One batched forward for all states; returns [(move, prob), ...] per state
        renormalised over the given (default: legal) moves (policy.py:44-79)."""
        n = len(states)
        if n == 0:
            return []
        size = states[0].size
        if any(st.size != size for st in states):
            raise ValueError("all states must have the same size")
        planes = self.preprocessor.states_to_uint8(states)
        probs = self.forward(planes)
        moves_lists = moves_lists or [st.get_legal_moves() for st in states]
        return [self._select(probs[i], moves_lists[i], size) for i in range(n)]

    def eval_state(self, state, moves=None):
        return self.batch_eval_state([state], [moves] if moves is not None else None)[0]

    @staticmethod
    def _select(dist, moves, size):
        if not moves:
            return []
        idx = [flatten_idx(m, size) for m in moves]
        d = dist[idx].astype(np.float64)
        s = d.sum()
        d = d / s if s > 0 else np.full(len(idx), 1.0 / len(idx))
        return list(zip(moves, d))


class CNNValue(_NetWrapper):
    """Value network (reference value.py): state -> expected outcome in [-1, 1]
    for the player to move."""

    _net_cls = ValueNet

    def __init__(self, feature_list: Sequence[str] = VALUE_FEATURES, device=None, **kwargs):
        super().__init__(feature_list, device=device, **kwargs)

    def _make_engine(self):
        return make_value_inference(self.model, self.device, **self._engine_kw())

    def forward(self, planes) -> np.ndarray:
        planes = np.asarray(planes).astype(np.uint8, copy=False)
        return self.engine.evaluate(planes).float().cpu().numpy()

    def batch_eval_state(self, states) -> List[float]:
        if not states:
            return []
        return [float(v) for v in self.forward(self.preprocessor.states_to_uint8(states))]

    def eval_state(self, state) -> float:
        return self.batch_eval_state([state])[0]
