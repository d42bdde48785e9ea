"""Training-position datasets (HDF5 schema of SURVEY.md §2.6).

``PositionDataset`` serves minibatches of (uint8 planes, int32 move targets)
on the training device.  Two residency modes:

* device-resident (default when it fits the budget): the whole ``states``
  array is copied to HBM once and batches are gathered on the GPU — the
  reference's per-sample host generator (supervised_policy_trainer.py:18-40)
  disappears from the step entirely.  288 GB of HBM per MI355X holds ~16 M
  positions of 48 planes; a node's 8 GPUs hold a full KGS-size dataset when
  each rank keeps only its shard.
* host-streamed: memory-mapped contiguous states, batch rows gathered into a
  pinned buffer and copied asynchronously.

The reference generator's data race (it mutated yielded buffers while Keras'
prefetch thread held them) does not exist here: each batch is a
fresh device tensor produced on the compute stream.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ..io.h5lite import H5File


class PositionDataset(object):
    def __init__(self, path: str, device=None, resident: str = "auto", budget_gb: float = 64.0):
        self.path = path
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.f = H5File(path)
        ds = self.f["states"]
        self.shape = ds.shape
        self.n, self.planes, self.size = ds.shape[0], ds.shape[1], ds.shape[2]
        acts = np.asarray(self.f["actions"].read()).astype(np.int64)
        self.targets_np = (acts[:, 0] * self.size + acts[:, 1]).astype(np.int32)
        self.features = [x.decode() for x in self.f.attrs["features"]] if "features" in self.f.attrs else None
        nbytes = int(np.prod(self.shape))
        fits = nbytes <= budget_gb * (1 << 30)
        self.resident = (resident == "yes") or (resident == "auto" and fits)
        self._states_np = ds.read()  # memmap view for contiguous data, decoded array for chunked
        if self.resident:
            self.states = torch.from_numpy(np.array(self._states_np, copy=True)).to(self.device)
            self.targets = torch.from_numpy(self.targets_np).to(self.device)
        else:
            self.states = None
            self.targets = None
            self._pin = None

    def __len__(self):
        return self.n

    def batch(self, idx: np.ndarray) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.resident:
            it = torch.from_numpy(np.asarray(idx, dtype=np.int64)).to(self.device, non_blocking=True)
            return self.states.index_select(0, it), self.targets.index_select(0, it)
        order = np.argsort(idx)
        rows = np.empty((len(idx),) + self.shape[1:], np.uint8)
        rows[order] = self._states_np[np.asarray(idx)[order]]
        t = torch.from_numpy(rows)
        tg = torch.from_numpy(self.targets_np[np.asarray(idx)])
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
            tg = tg.pin_memory().to(self.device, non_blocking=True)
        return t, tg

    def close(self):
        self.f.close()
