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

import collections
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
        backend, not enabled, or the library / communicator unavailable).

        Opt-in (``GARFIELD_DIRECT_RCCL=1``): the point-to-point exchange straight from the
        exchange rows and the staged next forward it enables have run on one GPU only (the
        one-rank test ``tests/test_rccl_gpu.py`` and the gloo contract rehearsals), never over
        xGMI between GPUs, so multi-rank jobs default to torch.distributed's packed
        ``all_to_all_single`` and the one-graph step."""
        if not direct_enabled() or not dist.is_initialized():
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

    def exchange(self, sends: list, to: list, recvs: list, frm: list, stream) -> None:
        """One group of ncclSend(sends[i] -> rank to[i]) / ncclRecv(recvs[i] <- rank frm[i]);
        transfers between one pair of ranks match in issue order."""
        if not sends and not recvs:   # one rank: nothing leaves
            return
        self._C.rccl_exchange(self.comm, sends, to, recvs, frm, self.world, stream.cuda_stream)

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor, stream) -> None:
        """recv = [world, *send.shape] flat; in place when send is recv's own rank block."""
        self._C.rccl_all_gather(self.comm, send, recv, self.world, stream.cuda_stream)

    def all_reduce_sum(self, t: torch.Tensor, stream) -> None:
        self._C.rccl_all_reduce_sum(self.comm, t, t, stream.cuda_stream)


# --------------------------------------------------------------------------- #
# The same call contract over torch.distributed, for multi-rank CPU rehearsals


class GlooDirect:
    """``DirectRCCL``'s exact call contract carried by torch.distributed (gloo on the CPU), so
    the multi-rank CPU tests run every ``self._rccl is not None`` branch of the exchange
    (``sharded.py``) that 8 MI355X will run, and check its layout assumptions:

    * ``all_to_all(send, recv)``: flat, contiguous, equal sizes; chunk r of ``send`` goes to
      rank r, chunk r of ``recv`` comes from rank r (``ncclAllToAll``);
    * ``all_gather(send, recv)``: ``recv`` = world x ``send``; when ``send`` overlaps ``recv`` it
      must be EXACTLY recv's own rank block (RCCL's in-place form), anything else is refused;
    * ``all_reduce_sum(t)``: in place;
    * ``exchange(sends, to, recvs, frm)``: one group of point-to-point transfers; every buffer
      flat and contiguous, no transfer to or from this rank itself, no receive buffer
      overlapping another buffer, and the sends to a peer pair up in order with that peer's
      receives (sizes checked against the peer's actual receives).

    ``calls`` counts the collectives by kind (the tests assert the per-step pattern)."""

    def __init__(self, world: int, rank: int):
        self.world = int(world)
        self.rank = int(rank)
        self.calls = collections.Counter()

    @staticmethod
    def _span(t: torch.Tensor):
        a = t.data_ptr()
        return a, a + t.numel() * t.element_size()

    def _overlap(self, a: torch.Tensor, b: torch.Tensor) -> bool:
        (a0, a1), (b0, b1) = self._span(a), self._span(b)
        return a0 < b1 and b0 < a1

    def all_to_all(self, send: torch.Tensor, recv: torch.Tensor, stream=None) -> None:
        if not (send.is_contiguous() and recv.is_contiguous() and send.dim() == 1 and recv.dim() == 1):
            raise ValueError("direct all_to_all: flat contiguous buffers")
        if send.numel() != recv.numel() or send.dtype != recv.dtype or send.numel() % self.world:
            raise ValueError("direct all_to_all: equal sizes divisible by the world size")
        if self._overlap(send, recv):
            raise ValueError("direct all_to_all: send and recv overlap")
        self.calls["all_to_all"] += 1
        dist.all_to_all_single(recv, send)

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor, stream=None) -> None:
        if not (send.is_contiguous() and recv.is_contiguous()):
            raise ValueError("direct all_gather: contiguous buffers")
        if recv.numel() != send.numel() * self.world or send.dtype != recv.dtype:
            raise ValueError("direct all_gather: output must be world x input")
        if self._overlap(send, recv):
            own = recv.data_ptr() + self.rank * send.numel() * send.element_size()
            if send.data_ptr() != own:
                raise ValueError("direct all_gather: an input inside the output must be this rank's block")
            send = send.clone()      # gloo refuses aliasing; RCCL reads its own block in place
            self.calls["all_gather_inplace"] += 1
        else:
            self.calls["all_gather"] += 1
        dist.all_gather_into_tensor(recv, send)

    def all_reduce_sum(self, t: torch.Tensor, stream=None) -> None:
        if not t.is_contiguous():
            raise ValueError("direct all_reduce: contiguous buffer")
        self.calls["all_reduce"] += 1
        dist.all_reduce(t)

    def exchange(self, sends: list, to: list, recvs: list, frm: list, stream=None) -> None:
        if len(sends) != len(to) or len(recvs) != len(frm):
            raise ValueError("direct exchange: one peer per buffer")
        for t, p in [*zip(sends, to), *zip(recvs, frm)]:
            if not (t.is_contiguous() and t.dim() == 1):
                raise ValueError("direct exchange: flat contiguous buffers")
            if not 0 <= p < self.world or p == self.rank:
                raise ValueError(f"direct exchange: peer {p} (the own shard never moves)")
        for i, r in enumerate(recvs):
            for t in [*sends, *recvs[:i]]:
                if self._overlap(r, t):
                    raise ValueError("direct exchange: a receive buffer overlaps another buffer")
        # the sizes each peer will send, checked against the receives posted for it (in order)
        mine = {p: [int(t.numel()) for t, q in zip(sends, to) if q == p] for p in range(self.world)}
        table = [None] * self.world
        dist.all_gather_object(table, mine)
        for p in range(self.world):
            if p != self.rank and table[p][self.rank] != [int(t.numel()) for t, q in zip(recvs, frm) if q == p]:
                raise ValueError(f"direct exchange: rank {p}'s sends do not match the receives posted for it")
        self.calls["exchange"] += 1
        ops = [dist.P2POp(dist.isend, t, p) for t, p in zip(sends, to)]
        ops += [dist.P2POp(dist.irecv, t, p) for t, p in zip(recvs, frm)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()


_OVERRIDE = None


def direct_enabled() -> bool:
    return os.environ.get("GARFIELD_DIRECT_RCCL", "0") == "1"


def set_direct_backend(factory) -> None:
    """``factory(world, rank)`` -> the direct backend every ``ShardedAggregator`` built next
    uses at world > 1 (e.g. ``GlooDirect`` in the CPU rehearsals); None restores the default
    (``DirectRCCL`` on RCCL process groups)."""
    global _OVERRIDE
    _OVERRIDE = factory


def direct_backend(world: int, rank: int, side: bool, world1: bool = False):
    """The direct backend of a sharded exchange: the override when set, else DirectRCCL when the
    exchange has its own comm stream and several ranks (``world1``: also on one rank, the
    test/trace run of the multi-rank call sequence)."""
    if world <= 1 and not world1:
        return None
    if _OVERRIDE is not None:
        return _OVERRIDE(world, rank)
    return DirectRCCL.create() if side else None
