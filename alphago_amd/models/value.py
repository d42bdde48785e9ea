"""Reference module path ``AlphaGo/models/value.py``: the paper's value-network
constants and the ``value_trainer`` class.

The reference builds the Keras model (value.py:12-31) and leaves
``get_samples`` / ``train`` as TODOs (value.py:33-39).  Here the model is the
``ValueNet`` of ``models/nets.py`` (49 planes, 5x5 + 11 x 3x3 convs of K
filters, 1x1 head, Dense(256), Dense(1, tanh)), ``get_samples`` draws
minibatches uniformly at random from self-play positions, and ``train`` runs
the HIP training engine (MSE; the CLI's Adam 3e-4 defaults) -- the same path as
``python -m alphago_amd.cli train-value`` (``train/value.py``).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from .nets import ValueNet

### Parameters obtained from paper ###
K = 152                        # depth of convolutional layers
LEARNING_RATE = .003           # initial learning rate
DECAY = 8.664339379294006e-08  # rate of exponential learning_rate decay


class value_trainer:  # noqa: N801 - reference class name
    """Value-network trainer on (states, outcomes) arrays: states (N, 49, S, S)
    uint8 planes, outcomes (N,) in {-1, 0, 1} for the player to move."""

    def __init__(self, states: Optional[np.ndarray] = None, outcomes: Optional[np.ndarray] = None,
                 minibatch: int = 32, device=None, seed: int = 0, **net_kwargs):
        kw = dict(input_dim=49, filters_per_layer=K, layers=12, dense=256)
        kw.update(net_kwargs)
        self.model = ValueNet(**kw)
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda" if torch.cuda.is_available() else "cpu")
        self.minibatch = minibatch
        self.states, self.outcomes = states, outcomes
        self.rng = np.random.default_rng(seed)
        self._trainer = None

    def get_samples(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        """Non-terminating generator of minibatches drawn uniformly at random
        (the reference's TODO, value.py:33-35)."""
        if self.states is None or self.outcomes is None:
            raise ValueError("value_trainer needs states and outcomes to sample from")
        n = len(self.outcomes)
        while True:
            idx = self.rng.integers(0, n, self.minibatch)
            x = torch.from_numpy(np.ascontiguousarray(self.states[idx], dtype=np.uint8)).to(self.device)
            z = torch.from_numpy(np.asarray(self.outcomes[idx], dtype=np.float32)).to(self.device)
            yield x, z

    def train(self, steps: int = 100, learning_rate: Optional[float] = None, decay: Optional[float] = None,
              backend: str = "auto", optimizer: Optional[str] = None) -> float:
        """Run ``steps`` optimizer steps (value.py:37-39 TODO); returns the mean MSE of the last step.

        Defaults are the ``train-value`` CLI's (train/value.py DEFAULT_OPTIMIZER / DEFAULT_LR): Keras 1.0
        Adam at 3e-4 with no decay on the reference's uniform init.  The paper's SGD(0.003, DECAY) on that
        init leaves a 12-layer trunk at the constant predictor (profiles/r4, profiles/r5); it stays
        available as ``optimizer="sgd"`` (then learning_rate / decay default to LEARNING_RATE / DECAY)."""
        from ..train.engine import make_value_trainer
        from ..train.value import DEFAULT_LR, DEFAULT_OPTIMIZER

        optimizer = optimizer or DEFAULT_OPTIMIZER
        if learning_rate is None:
            learning_rate = DEFAULT_LR[optimizer]
        if decay is None:
            decay = 0.0 if optimizer == "adam" else DECAY
        if self._trainer is None:
            self.model.to(self.device)
            self._trainer = make_value_trainer(self.model, self.minibatch, learning_rate, decay, backend=backend,
                                               device=self.device, optimizer=optimizer)
        gen = self.get_samples()
        loss = 0.0
        for _ in range(steps):
            x, z = next(gen)
            sym = torch.from_numpy(self.rng.integers(0, 8, self.minibatch).astype(np.int32)).to(self.device)
            lsum, _ = self._trainer.step(x, z, sym)
            loss = float(lsum) / self.minibatch
        return loss
