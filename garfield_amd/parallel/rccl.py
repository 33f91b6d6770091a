"""RCCL collectives enqueued straight onto a stream of ours (no torch stream hop).

``torch.distributed`` (ProcessGroupNCCL) runs each collective on an internal stream
that waits, with a HIP event, on the caller's current stream. On ROCm 7 / MI355X any
such pending cross-stream event wait slows a HIP graph replaying meanwhile by ~1-1.5
us per kernel (``signals.py``, ``profiles/r3/probe_cross_stream.log``) -- during the
overlapped exchange that would be the whole backward. ``DirectRCCL`` calls torch's
own librccl on torch's own communicator (``ProcessGroupNCCL._comm_ptr()``) with the
exchange's comm stream, which follows the main stream through device-side counters:
the kernels simply run in that stream's order. Results come back to the main stream
through an event the MAIN stream waits on (that direction costs nothing measurable).

Every rank issues the same collectives in the same order (the engine's step is
deterministic), which is all RCCL requires; torch's collectives on the same
communicator (barriers, checkpoints) are ordered after ours by the callers
(``ShardedAggregator.quiesce``).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from garfield_amd import _native


class DirectRCCL:
    def __init__(self, comm: int, world: int):
        self._C = _native.native()
        self.comm = int(comm)
        self.world = int(world)

    @classmethod
    def create(cls, group=None) -> "DirectRCCL | None":
        """The direct path for the default (or given) NCCL process group, or None (another
        backend, ``GARFIELD_DIRECT_RCCL=0``, or the library / communicator unavailable)."""
        if os.environ.get("GARFIELD_DIRECT_RCCL", "1") == "0" or not dist.is_initialized():
            return None
        pg = group or dist.distributed_c10d._get_default_group()
        if dist.get_backend(pg) != "nccl":
            return None
        try:
            backend = pg._get_backend(torch.device("cuda"))
            comm = backend._comm_ptr()
        except Exception:
            return None
        if not comm:
            return None
        C = _native.native()
        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not (os.path.exists(lib) and C.rccl_load(lib)):
            return None
        return cls(comm, dist.get_world_size(pg))

    def all_to_all(self, send: torch.Tensor, recv: torch.Tensor, stream) -> None:
        self._C.rccl_all_to_all(self.comm, send, recv, self.world, stream.cuda_stream)

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor, stream) -> None:
        """recv = [world, *send.shape] flat; in place when send is recv's own rank block."""
        self._C.rccl_all_gather(self.comm, send, recv, self.world, stream.cuda_stream)

    def all_reduce_sum(self, t: torch.Tensor, stream) -> None:
        self._C.rccl_all_reduce_sum(self.comm, t, t, stream.cuda_stream)
