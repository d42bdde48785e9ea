"""Training-position datasets (HDF5 schema of SURVEY.md §2.6).

``PositionDataset`` serves minibatches of (uint8 planes, int32 move targets)
on the training device.  Each rank opens the file with the global row ids it
owns (``rows``: its shard of the shuffled train/val permutation, see
``shard_rows``), so a rank never holds another rank's positions — host RAM and
HBM per rank are ~N/world rows, and a node's 8 x 288 GB of HBM holds a full
KGS-size dataset.  Batches are addressed by *local* position (index into
``rows``).  Two residency modes:

* device-resident (default when the shard fits the budget): the shard's rows
  are decoded once (chunk-sliced for chunked/LZF files: each chunk that holds
  a shard row is decoded once, one block of chunks at a time, never the whole
  file) and copied to HBM; batches are gathered on the GPU — the reference's
  per-sample host generator (supervised_policy_trainer.py:18-40) disappears
  from the step.
* host-streamed: rows are read on demand (memory-mapped for contiguous files,
  a small LRU of decoded chunks for chunked files).  ``prefetch()`` runs a
  worker thread that gathers the rows of upcoming batches into a ring of
  pinned host buffers and copies them to preallocated device slots on a
  dedicated copy stream; the consumer's stream waits on the copy's event, so
  neither the gather nor the H2D copy sits on the training step's critical
  path.  With a chunked file the shard is visited in block-shuffled order
  (``block_shuffle``: chunks in random order, rows shuffled within a window of
  chunks) so each chunk is decoded about once per pass instead of once per row.

The reference generator's data race (it mutated yielded buffers while Keras'
prefetch thread held them) does not exist here: a slot is handed to
the consumer only after its copy event, and refilled only after the consumer's
stream has passed the step that read it.
"""
from __future__ import annotations

import os
import queue
import threading
from collections import OrderedDict
from typing import Iterable, Iterator, Optional, Tuple

import numpy as np
import torch

from ..io.h5lite import H5File


def shard_rows(idx: np.ndarray, rank: int, world: int) -> np.ndarray:
    """This rank's fixed partition of a (shuffled) index array: idx[rank::world]."""
    return np.asarray(idx, np.int64)[rank::world]


def block_shuffle(rows: np.ndarray, chunk_rows: int, seed: int, window: int = 16) -> np.ndarray:
    """Reorder ``rows`` so that consecutive positions stay within a window of
    ``window`` file chunks: chunks in random order, rows shuffled inside each
    window.  Every row is kept exactly once."""
    rows = np.asarray(rows, np.int64)
    if len(rows) == 0 or chunk_rows <= 0:
        return rows
    rng = np.random.default_rng(seed)
    chunk = rows // chunk_rows
    uniq = np.unique(chunk)
    order = rng.permutation(len(uniq))
    rank_of_chunk = np.empty(int(uniq.max()) + 1, np.int64)
    rank_of_chunk[uniq[order]] = np.arange(len(uniq))
    key = rank_of_chunk[chunk]
    srt = rows[np.argsort(key, kind="stable")]
    ksrt = np.sort(key)
    out = np.empty_like(srt)
    for w0 in range(0, len(uniq), window):
        sel = np.flatnonzero((ksrt >= w0) & (ksrt < w0 + window))
        out[sel] = srt[sel][rng.permutation(len(sel))]
    return out


class _ChunkCache(object):
    """LRU of decoded chunks of one chunked dataset, kept in one preallocated
    slot array so a batch gather is a single ``np.take`` (GIL released).

    ``gather`` holds a lock for its whole duration: the prefetch worker and the
    main thread (validation batches) share one cache, and an unlocked gather
    could evict or overwrite a slot the other thread is about to read."""

    def __init__(self, ds, capacity: int, threads: int):
        self.lock = threading.Lock()
        self.ds, self.cap, self.threads = ds, max(1, capacity), threads
        self.cr = ds.chunk_rows
        self.slots = np.zeros((self.cap * self.cr,) + tuple(ds.shape[1:]), ds.dtype)  # touched once
        self.slot_of: "OrderedDict[int, int]" = OrderedDict()  # chunk id -> slot, LRU order
        self.free = list(range(self.cap))

    def gather(self, rows: np.ndarray, out: np.ndarray) -> None:
        with self.lock:
            self._gather(rows, out)

    def _gather(self, rows: np.ndarray, out: np.ndarray) -> None:
        cids = rows // self.cr
        uniq = np.unique(cids)
        if len(uniq) > self.cap:  # batch wider than the cache: grow it
            extra = len(uniq) - self.cap
            self.slots = np.concatenate([self.slots, np.zeros((extra * self.cr,) + self.slots.shape[1:],
                                                              self.slots.dtype)])
            self.free += list(range(self.cap, self.cap + extra))
            self.cap += extra
        for c in uniq:
            if int(c) in self.slot_of:
                self.slot_of.move_to_end(int(c))
        need = [int(c) for c in uniq if int(c) not in self.slot_of]
        if need:
            keep = set(int(c) for c in uniq)
            while len(self.free) < len(need):
                for old in self.slot_of:
                    if old not in keep:
                        self.free.append(self.slot_of.pop(old))
                        break
            dst = [self.free.pop() for _ in need]
            self.ds.read_chunks(need, self.threads, out=self.slots, slots=dst)  # decoded in place
            for c, sl in zip(need, dst):
                self.slot_of[c] = sl
        slot = np.fromiter((self.slot_of[int(c)] for c in cids), np.int64, len(cids))
        np.take(self.slots, slot * self.cr + rows % self.cr, axis=0, out=out)


class PositionDataset(object):
    def __init__(self, path: str, device=None, resident: str = "auto", budget_gb: float = 64.0,
                 rows: Optional[np.ndarray] = None, threads: int = 0, cache_chunks: int = 64,
                 targets: str = "actions"):
        self.path = path
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.f = H5File(path)
        ds = self.f["states"]
        self._ds = ds
        self.shape = ds.shape
        self.n, self.planes, self.size = ds.shape[0], ds.shape[1], ds.shape[2]
        self.row_shape = tuple(ds.shape[1:])
        self.threads = threads or min(16, os.cpu_count() or 8)  # LZF decode threads
        if targets == "actions":  # move (x, y) -> flat index x*S+y (util.py:6-8)
            acts = np.asarray(self.f["actions"].read()).astype(np.int64)
            self._targets_all = (acts[:, 0] * self.size + acts[:, 1]).astype(np.int32)
        elif targets == "outcomes":  # value-network regression targets z in {-1, 0, 1}
            self._targets_all = np.asarray(self.f["outcomes"].read()).astype(np.float32)
        else:
            raise ValueError("targets must be 'actions' or 'outcomes'")
        self.features = [x.decode() for x in self.f.attrs["features"]] if "features" in self.f.attrs else None
        self.chunked = ds.chunked
        self.chunk_rows = ds.chunk_rows if ds.chunked else 0
        self.rows = np.arange(self.n, dtype=np.int64) if rows is None else np.asarray(rows, np.int64)
        if len(self.rows) and (self.rows.min() < 0 or self.rows.max() >= self.n):
            raise IndexError("row ids outside [0, %d)" % self.n)
        self.targets_np = self._targets_all[self.rows]
        nbytes = len(self.rows) * int(np.prod(self.row_shape))
        fits = nbytes <= budget_gb * (1 << 30)
        self.resident = (resident == "yes") or (resident == "auto" and fits)
        self._cache = _ChunkCache(ds, cache_chunks, self.threads) if self.chunked and not self.resident else None
        self._stage = None
        if self.resident:
            host = self._load_rows(self.rows)
            self.states = torch.from_numpy(host).to(self.device)
            self.targets = torch.from_numpy(self.targets_np).to(self.device)
        else:
            self.states = None
            self.targets = None

    # ------------------------------------------------------------ host reads
    def _load_rows(self, rows: np.ndarray) -> np.ndarray:
        """Rows in the given order; chunked files are decoded a block of chunks
        at a time, each chunk holding a requested row decoded exactly once."""
        out = np.empty((len(rows),) + self.row_shape, np.uint8)
        if not self.chunked:
            mm = self._ds.read()
            order = np.argsort(rows, kind="stable")
            for s in range(0, len(rows), 65536):
                sel = order[s:s + 65536]
                out[sel] = mm[rows[sel]]
            return out
        cr = self.chunk_rows
        order = np.argsort(rows, kind="stable")
        srows = rows[order]
        cids = srows // cr
        uniq, first = np.unique(cids, return_index=True)
        bounds = list(first) + [len(srows)]
        per_block = 256
        block = np.zeros((min(per_block, len(uniq)) * cr,) + self.row_shape, np.uint8)  # reused
        for b0 in range(0, len(uniq), per_block):
            ids = uniq[b0:b0 + per_block]
            self._ds.read_chunks(ids.tolist(), self.threads, out=block)
            lo, hi = bounds[b0], bounds[min(b0 + per_block, len(uniq))]
            rel = np.searchsorted(ids, cids[lo:hi]) * cr + srows[lo:hi] % cr
            out[order[lo:hi]] = block[rel]
        return out

    def _gather_host(self, pos: np.ndarray, out: np.ndarray) -> None:
        rows = self.rows[pos]
        if self.chunked:
            self._cache.gather(rows, out)
        else:
            np.take(self._ds.read(), rows, axis=0, out=out)

    # ------------------------------------------------------------- batches
    def __len__(self):
        return len(self.rows)

    def batch(self, pos: np.ndarray) -> Tuple[torch.Tensor, torch.Tensor]:
        """Synchronous batch of local positions."""
        pos = np.asarray(pos, np.int64)
        if self.resident:
            it = torch.from_numpy(pos).to(self.device, non_blocking=True)
            return self.states.index_select(0, it), self.targets.index_select(0, it)
        n = len(pos)
        if self._stage is None or self._stage[0].shape[0] < n:
            pin = self.device.type == "cuda"
            self._stage = (torch.empty((n,) + self.row_shape, dtype=torch.uint8, pin_memory=pin),
                           torch.empty((n,), dtype=torch.from_numpy(self.targets_np[:0]).dtype, pin_memory=pin))
        hx, ht = self._stage[0][:n], self._stage[1][:n]
        self._gather_host(pos, hx.numpy())
        ht.numpy()[:] = self.targets_np[pos]
        if self.device.type == "cuda":
            x, t = hx.to(self.device, non_blocking=True), ht.to(self.device, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()  # the staging buffer is reused next call
            return x, t
        return hx.clone(), ht.clone()

    def prefetch(self, batches: Iterable[np.ndarray], batch_size: int, depth: int = 3) -> "Prefetcher":
        return Prefetcher(self, batches, batch_size, depth)

    def close(self):
        self.f.close()


class Prefetcher(object):
    """Iterator of device batches fed by a worker thread (see module doc).
    A returned batch stays valid until the next ``__next__`` call."""

    def __init__(self, ds: PositionDataset, batches: Iterable[np.ndarray], batch_size: int, depth: int = 3):
        self.ds, self.B, self.depth = ds, batch_size, max(2, depth)
        dev = ds.device
        self.cuda = dev.type == "cuda"
        shape = (batch_size,) + ds.row_shape
        tdt = torch.from_numpy(ds.targets_np[:0]).dtype
        self.hx = [torch.empty(shape, dtype=torch.uint8, pin_memory=self.cuda) for _ in range(self.depth)]
        self.ht = [torch.empty((batch_size,), dtype=tdt, pin_memory=self.cuda) for _ in range(self.depth)]
        if self.cuda:
            self.dx = [torch.empty(shape, dtype=torch.uint8, device=dev) for _ in range(self.depth)]
            self.dt = [torch.empty((batch_size,), dtype=tdt, device=dev) for _ in range(self.depth)]
            self.copy_stream = torch.cuda.Stream(dev)
            self.copied = [torch.cuda.Event() for _ in range(self.depth)]
            self.consumed = [None] * self.depth
        self.free: "queue.Queue[int]" = queue.Queue()
        for i in range(self.depth):
            self.free.put(i)
        self.ready: "queue.Queue" = queue.Queue()
        self._it = iter(batches)
        self._held = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._work, name="position-prefetch", daemon=True)
        self._thread.start()

    def _work(self):
        try:
            for pos in self._it:
                pos = np.asarray(pos, np.int64)
                if len(pos) != self.B:
                    raise ValueError("prefetch batches must have %d rows" % self.B)
                i = self.free.get()
                if self._stop.is_set():
                    return
                if self.cuda and self.consumed[i] is not None:
                    self.consumed[i].synchronize()  # the step that read slot i has run: host + device buffers free
                self.ds._gather_host(pos, self.hx[i].numpy())
                self.ht[i].numpy()[:] = self.ds.targets_np[pos]
                if self.cuda:
                    with torch.cuda.stream(self.copy_stream):
                        self.dx[i].copy_(self.hx[i], non_blocking=True)
                        self.dt[i].copy_(self.ht[i], non_blocking=True)
                        self.copied[i].record(self.copy_stream)
                self.ready.put(i)
        except BaseException as e:  # surfaced in the consumer
            self.ready.put(e)
            return
        self.ready.put(None)

    def _release(self):
        if self._held is not None:
            i = self._held
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.ds.device))
                self.consumed[i] = ev
            self._held = None
            self.free.put(i)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        return self

    def __next__(self) -> Tuple[torch.Tensor, torch.Tensor]:
        self._release()
        i = self.ready.get()
        if i is None:
            raise StopIteration
        if isinstance(i, BaseException):
            raise i
        self._held = i
        if self.cuda:
            torch.cuda.current_stream(self.ds.device).wait_event(self.copied[i])
            return self.dx[i], self.dt[i]
        return self.hx[i].clone(), self.ht[i].clone()

    def close(self):
        self._stop.set()
        self._release()
        for _ in range(self.depth):
            self.free.put(0)
        self._thread.join(timeout=10)
