"""Process-group setup and gradient collectives (RCCL over xGMI on MI355X).

One process per GPU.  ``init_from_env`` reads RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT (torchrun convention) and initialises
``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm) when a GPU is
present, ``gloo`` otherwise (CPU tests).

The reference has no distributed machinery at all; data
parallelism is new here.  Gradients live in one flat fp32 buffer laid out in
*forward* layer order, so the buckets that become ready during backward
(last layers first) are contiguous slices: each bucket is all-reduced as soon
as its wgrad reductions are enqueued, on the RCCL stream, overlapping the
remaining dgrad/wgrad kernels.  Bucket size defaults to ~4 MiB — a ring
all-reduce over xGMI point-to-point links is per-link bound and 8-16 MB of
total gradients per step gives only a few buckets, each large enough to use
the links but small enough to start early.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    forced: bool = False  # ALPHAGO_AMD_FORCE_DIST=1: a process group even at world 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.forced


_ENV: Optional[DistEnv] = None


def init_from_env(device: str = "auto", timeout_s: float = 600.0) -> DistEnv:
    """Initialise (once) from torchrun-style environment variables."""
    global _ENV
    if _ENV is not None:
        return _ENV
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
    if use_gpu:
        ndev = max(1, torch.cuda.device_count())
        torch.cuda.set_device(local % ndev)
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    backend = "none"
    # ALPHAGO_AMD_FORCE_DIST=1 creates the process group at world 1 too, so every collective of
    # the data-parallel path (broadcast, bucketed async all-reduce, barrier, metric reductions)
    # runs through RCCL on a one-GPU box: RCCL refuses two ranks on one device
    # (profiles/r2_rccl_same_gpu.md).
    forced = world == 1 and os.environ.get("ALPHAGO_AMD_FORCE_DIST", "0") == "1"
    if world > 1 or forced:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = os.environ.get("ALPHAGO_AMD_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        kw = {}
        if use_gpu and backend == "nccl":
            kw["device_id"] = dev
        tmo = datetime.timedelta(seconds=timeout_s)
        attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if attempt > 0:
            # torchrun --max-restarts reuses the rendezvous store across
            # attempts; namespace this attempt's keys so the new group does
            # not pick up the dead group's peer addresses.
            store, _, _ = next(dist.rendezvous("env://", rank, world, timeout=tmo))
            store = dist.PrefixStore("attempt%d/" % attempt, store)
            dist.init_process_group(backend=backend, store=store, rank=rank, world_size=world, timeout=tmo, **kw)
        else:
            dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=tmo, **kw)
    _ENV = DistEnv(rank=rank, local_rank=local, world_size=world, backend=backend, device=dev, forced=forced)
    return _ENV


def env() -> DistEnv:
    return _ENV or DistEnv()


def shutdown() -> None:
    global _ENV
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _ENV = None


def live_backend() -> str:
    """The initialised process group's backend as torch reports it ("nccl" = RCCL on ROCm), or "none"."""
    if dist.is_available() and dist.is_initialized():
        return str(dist.get_backend())
    return "none"


def live_world_size() -> int:
    if dist.is_available() and dist.is_initialized():
        return int(dist.get_world_size())
    return 1


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if env().backend == "nccl":
            dist.barrier(device_ids=[env().device.index])
        else:
            dist.barrier()


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized():
        dist.broadcast(t, src)
    return t


def all_reduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t)
    return t


def all_reduce_max(value: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return value
    dev = env().device if env().backend == "nccl" else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_object(obj):
    """List of every rank's ``obj`` (rank order); ``[obj]`` when not distributed."""
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def make_buckets(segments: Sequence[Tuple[int, int]], bucket_bytes: int = 4 << 20,
                 elem_bytes: int = 4, last_alone: bool = False) -> List[Tuple[int, int, List[int]]]:
    """Group per-layer flat segments (offset, numel) — given in *backward*
    order — into contiguous buckets.  Returns [(offset, numel, [segment ids])].
    ``last_alone``: the last segment (the first layer, whose gradient is ready only at
    the very end of the backward) gets a bucket of its own, so the bucket before it is
    launched one layer earlier and overlaps the final dgrad + wgrad; only the small
    first-layer all-reduce is left exposed."""
    buckets: List[Tuple[int, int, List[int]]] = []
    cur_lo = cur_hi = None
    cur_ids: List[int] = []
    for sid, (off, n) in enumerate(segments):
        lo, hi = off, off + n
        tail = last_alone and sid == len(segments) - 1 and len(segments) > 1
        if cur_ids and (tail or (hi - lo + (cur_hi - cur_lo)) * elem_bytes > bucket_bytes):
            buckets.append((cur_lo, cur_hi - cur_lo, cur_ids))
            cur_ids, cur_lo, cur_hi = [], None, None
        if not cur_ids:
            cur_lo, cur_hi = lo, hi
        else:
            if hi != cur_lo and lo != cur_hi:
                raise ValueError("segments are not contiguous in backward order")
            cur_lo, cur_hi = min(cur_lo, lo), max(cur_hi, hi)
        cur_ids.append(sid)
    if cur_ids:
        buckets.append((cur_lo, cur_hi - cur_lo, cur_ids))
    return buckets


class BucketAllReducer:
    """Async per-bucket all-reduce of slices of a flat gradient buffer."""

    def __init__(self, flat: torch.Tensor, buckets):
        self.flat = flat
        self.buckets = buckets
        self.handles = []

    def launch(self, bucket_idx: int) -> None:
        if not (dist.is_available() and dist.is_initialized()):
            return
        off, n, _ = self.buckets[bucket_idx]
        self.handles.append(dist.all_reduce(self.flat[off:off + n], async_op=True))

    def wait(self) -> None:
        for h in self.handles:
            h.wait()
        self.handles = []


class CommProxy:
    """One-GPU stand-in for the bucketed all-reduce (same launch points, same waits): each bucket
    launches ``ops.comm_proxy`` on a high-priority side stream -- ``channels`` workgroups that read
    the bucket (the gradient is never modified) and hold their CUs for the modelled ring time
    ``latency_us + bytes * 2 (W-1) / W / busbw`` -- so the CU contention of an overlapped all-reduce
    can be measured without a second GPU (RCCL refuses two ranks on one device).

    Configured by ``ALPHAGO_AMD_COMM_PROXY=channels,busbw_GBps,world[,latency_us]``."""

    def __init__(self, flat: torch.Tensor, buckets, channels: int = 16, busbw_gbs: float = 300.0, world: int = 8,
                 latency_us: float = 15.0):
        from .. import ops
        self.ops = ops
        self.flat, self.buckets = flat, buckets
        self.channels = int(channels)
        self.factor = 2.0 * (world - 1) / world
        self.busbw = float(busbw_gbs) * 1e9
        self.latency_us = float(latency_us)
        n = max(b[1] for b in buckets) + 8
        self.scratch = torch.empty(n, dtype=torch.float32, device=flat.device)
        self.stream = torch.cuda.Stream(device=flat.device, priority=-1)
        self.launched = False

    @staticmethod
    def from_env(flat, buckets):
        spec = os.environ.get("ALPHAGO_AMD_COMM_PROXY", "")
        if not spec:
            return None
        v = [float(x) for x in spec.split(",")]
        return CommProxy(flat, buckets, int(v[0]), v[1] if len(v) > 1 else 300.0, int(v[2]) if len(v) > 2 else 8,
                         v[3] if len(v) > 3 else 15.0)

    def wire_us(self, bucket_idx: int) -> float:
        return self.latency_us + self.buckets[bucket_idx][1] * 4 * self.factor / self.busbw * 1e6

    def launch(self, bucket_idx: int) -> None:
        off, n, _ = self.buckets[bucket_idx]
        lo = off - off % 4  # 16-byte aligned float4 view (reads a few neighbours: read-only)
        hi = min(self.flat.numel(), (off + n + 3) // 4 * 4)
        hi = lo + (hi - lo) // 4 * 4
        ev = torch.cuda.current_stream(self.flat.device).record_event()
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            self.ops.comm_proxy(self.flat[lo:hi], self.scratch, self.channels, self.wire_us(bucket_idx))
        self.launched = True

    def wait(self) -> None:
        if self.launched:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)
            self.launched = False
