"""Process groups and collectives over RCCL (xGMI) / gloo.

Reference: the RPC pulls of ``garfieldpp/server.py`` (pickled model to every worker,
flat CPU gradient back, per worker per step) and the per-parameter-tensor
``dist.gather`` / ``dist.broadcast`` loops of ``applications/Garfield_CC/trainer.py:
55-207`` (gloo only, "NCCL does not support gather").

MI355X design (one process per GPU, ``backend="nccl"`` = RCCL):

* gradients travel as ONE flat bf16 row per logical worker, all-gathered with
  ``all_gather_into_tensor`` straight into the ``[n, d]`` buffer the GAR kernels
  read (no stacking copy; in-place: each rank's row already sits at its slot);
* a robust GAR needs every individual gradient, so an all-reduce is useless here;
  an all-gather over the xGMI full mesh receives from all 7 peers at once;
* role groups (parameter servers, workers, worker+servers) replace Garfield_CC's
  per-worker broadcast groups for the Byzantine-server mode.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    backend: str = "none"
    initialized_here: bool = False

    @property
    def is_distributed(self) -> bool:
        """Whether the engines issue their collectives: several ranks, or the one-rank RCCL
        rehearsal of the multi-rank step (``world1_collectives``)."""
        return collectives_on(self.world_size)

    def barrier(self) -> None:
        if self.is_distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


def init_distributed(backend: str | None = None, device: str | None = None, timeout_s: float = 1800.0) -> DistContext:
    """Initialise ``torch.distributed`` from the torchrun environment (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT). One process per GPU; RCCL when GPUs are present.

    Rehearsal knobs (multi-rank GPU code paths on a one-GPU box, where RCCL refuses
    two ranks on one device): ``GARFIELD_DIST_BACKEND`` overrides the backend (e.g.
    ``gloo``, which takes GPU tensors), ``GARFIELD_SHARE_GPU=1`` maps local rank r to
    device ``r % device_count``."""
    backend = backend or os.environ.get("GARFIELD_DIST_BACKEND") or None
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() if device is None else device.startswith("cuda")
    if use_cuda:
        idx = local % max(torch.cuda.device_count(), 1) if os.environ.get("GARFIELD_SHARE_GPU") == "1" else local
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
    else:
        dev = torch.device("cpu")
    backend = backend or ("nccl" if use_cuda else "gloo")
    ctx = DistContext(rank, world, local, dev, backend if world > 1 else "none")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        ctx.initialized_here = True
    elif world == 1 and world1_requested() and not dist.is_initialized():
        # a one-rank communicator (RCCL on a GPU) on which the world-1 run issues every
        # collective of the multi-rank step (world1_collectives)
        import socket

        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        kw = {"device_id": dev} if use_cuda else {}
        dist.init_process_group("nccl" if use_cuda else "gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                world_size=1, **kw)
        ctx.backend = "nccl" if use_cuda else "gloo"
        ctx.initialized_here = True
    return ctx


def world1_requested() -> bool:
    """``GARFIELD_COLL_WORLD1=1``: a one-rank job runs the multi-rank code path with real
    collectives on a one-rank process group instead of taking its world-1 shortcuts: the
    sharded step's packed all-to-all per bucket from the comm stream, partial-Gram all-gather,
    in-place weight all-gathers and BatchNorm-affine all-reduce; the unsharded slot
    all-gathers; the Byzantine-server broadcasts; the quorum engine's per-root groups. On
    one GPU this exercises every RCCL call pattern of the 8-GPU job (tests, traces)."""
    return os.environ.get("GARFIELD_COLL_WORLD1", "0") == "1"


def world1_collectives() -> bool:
    """``world1_requested()`` and a process group is initialised (of one rank)."""
    return world1_requested() and dist.is_available() and dist.is_initialized()


def collectives_on(world: int) -> bool:
    """Whether a job of ``world`` ranks issues its collectives (every multi-rank job; a
    one-rank job under ``GARFIELD_COLL_WORLD1=1`` with a one-rank process group)."""
    if world > 1:
        return dist.is_available() and dist.is_initialized()
    return world1_collectives()


def shutdown(ctx: DistContext) -> None:
    if ctx.initialized_here and dist.is_initialized():
        dist.destroy_process_group()


def gloo_backend(group=None) -> bool:
    """True when the collectives run on gloo (which rejects an input aliasing the output,
    on CPU and GPU tensors alike)."""
    return dist.is_initialized() and dist.get_backend(group) == "gloo"


def all_gather_rows(out_rows: torch.Tensor, rank: int, group=None, async_op: bool = False):
    """In-place all-gather of ``out_rows[rank]`` into every row of ``out_rows`` ([world, ld], contiguous).

    The output is passed flat (gloo requires it; RCCL does not care) and the input
    is this rank's own row, i.e. NCCL/RCCL's in-place all-gather form."""
    assert out_rows.is_contiguous()
    if gloo_backend(group):
        # gloo does not support the in-place form (input aliasing the output)
        return dist.all_gather_into_tensor(out_rows.view(-1), out_rows[rank].clone(), group=group,
                                           async_op=async_op)
    return dist.all_gather_into_tensor(out_rows.view(-1), out_rows[rank], group=group, async_op=async_op)


def broadcast_flat(t: torch.Tensor, src: int, group=None, async_op: bool = False):
    return dist.broadcast(t, src=src, group=group, async_op=async_op)


@dataclass
class RoleGroups:
    """Groups for the replicated-server (ByzSGD / GuanYu) topology: ranks
    ``[0, num_ps)`` are parameter servers, the others workers (the Garfield_CC
    convention, ``trainer.py:279,355-365``)."""

    num_ps: int
    world_size: int
    all: object = None
    ps: object = None
    workers: object = None

    @property
    def ps_ranks(self) -> list[int]:
        return list(range(self.num_ps))

    @property
    def worker_ranks(self) -> list[int]:
        return list(range(self.num_ps, self.world_size))


def make_role_groups(num_ps: int, world_size: int) -> RoleGroups:
    rg = RoleGroups(num_ps, world_size)
    if collectives_on(world_size):
        rg.all = dist.group.WORLD
        rg.ps = dist.new_group(rg.ps_ranks) if num_ps > 0 else None
        rg.workers = dist.new_group(rg.worker_ranks) if world_size > num_ps else None
    return rg
