"""Parameter server node (reference ``garfieldpp/server.py:58-305``).

Same constructor and methods as the reference; the RPC topology (``ps:i`` /
``worker:i`` / ``node:i`` names over ``torch.distributed.rpc``) is kept for API
compatibility. MI355X-side differences:

* the model and the optimizer live on the GPU (the reference keeps them on the
  CPU, "RPC is not supported on GPUs", ``server.py:89``); what travels over RPC is
  the reference-layout flat parameter vector, not a pickled ``nn.Module``;
* received gradients are packed into one aligned ``[n, d]`` device buffer, so the
  GAR (HIP kernels) reads them without stacking copies;
* "wait for the fastest k" uses a condition variable signalled by the RPC
  futures' callbacks (the reference sleep-polls every 10 ms, ``server.py:151-152``);
* ``compute_accuracy`` evaluates a snapshot replica (the reference deep-copies the
  live model in a thread while ``update_model`` mutates it — a race);
* ``world_size == 0`` builds a standalone server with no RPC (bug B6: Centralized).
"""
from __future__ import annotations

import copy
import logging
import threading

import torch
import torch.nn as nn

from garfield_amd.data.datasets import DatasetManager
from garfield_amd.runtime import tools
from garfield_amd.runtime.tools import _remote_method_async
from garfield_amd.utils.flat import FlatParams, padded

logger = logging.getLogger(__name__)


class _Quorum:
    """Collects up to n results from RPC futures; wait(k) returns once k arrived."""

    def __init__(self, n: int):
        self.items = [None] * n
        self.count = 0
        self.cv = threading.Condition()
        self.error = None

    def callback(self, slot: int, unpack):
        def cb(fut):
            try:
                val = unpack(fut.wait())
            except Exception as e:  # surface remote failures to the waiter
                with self.cv:
                    self.error = e
                    self.cv.notify_all()
                return
            with self.cv:
                self.items[slot] = val
                self.count += 1
                self.cv.notify_all()
        return cb

    def wait(self, k: int, timeout: float | None = None):
        with self.cv:
            ok = self.cv.wait_for(lambda: self.count >= k or self.error is not None, timeout=timeout)
            if self.error is not None and self.count < k:
                raise self.error
            if not ok:
                raise TimeoutError(f"only {self.count} of {k} replies arrived")
            return [x for x in self.items if x is not None]


class Server:
    """Byzantine-resilient parameter server."""

    def __init__(self, rank, world_size, num_workers, num_ps, byz_wrk, byz_ps, wrk_base_name, ps_base_name, batch,
                 model, dataset, optimizer, train_size=None, *args, device=None, register: bool = True,
                 rpc_timeout: float | None = None, **kwargs):
        self.device = torch.device(device) if device else (
            torch.device("cuda") if torch.cuda.device_count() > 0 else torch.device("cpu"))
        self.rank = rank
        self.world_size = world_size
        self.num_workers = num_workers
        self.byz_wrk = byz_wrk
        self.byz_ps = byz_ps
        self.num_ps = num_ps
        self.rpc_timeout = rpc_timeout
        self.model_name, self.dataset = model, dataset
        self.lock = threading.RLock()          # guards the model against concurrent RPC readers
        self._aggr_ready = threading.Event()
        self._latest = None
        if world_size > 0 and num_workers > 0:
            self.workers_types, self.workers_rref = self.get_rrefs(wrk_base_name, 0, num_workers, True)
        self.model = tools.select_model(model, self.device, dataset)
        self.flat = FlatParams(self.model, device=self.device, with_grad=True)
        if register:  # announce before fetching peer servers (they may fetch us concurrently)
            tools.register_server(self)
        manager = DatasetManager(dataset, batch * max(num_workers, 1), 1, 2, 1, train_size, device=self.device)
        self.test_set = manager.get_test_set()
        self.train_set = manager.get_train_set()
        self.optimizer = tools.select_optimizer(self.model, optimizer, *args, **kwargs)
        self._gbuf = None
        if world_size > 0 and num_ps > 0:
            self.ps_types, self.ps_rref = self.get_rrefs(ps_base_name, 0, num_ps, False)

    # ------------------------------------------------------------------ #

    def get_rrefs(self, base_name, base_id, num_nodes, worker=True):
        """RRefs to the remote worker/server singletons and their classes.

        The class is fetched by a remote ``type()`` call; the reference used
        ``type(rref.to_here())``, which pickles the whole remote node."""
        from torch.distributed.rpc import remote, rpc_sync

        rrefs = [remote(base_name + str(i), tools.get_worker if worker else tools.get_server)
                 for i in range(base_id, base_id + num_nodes)]
        types = [rpc_sync(r.owner(), tools._type_of, args=(r,)) for r in rrefs]
        return types, rrefs

    def _payload(self):
        """What workers receive: the reference-layout flat parameter vector (CPU)."""
        with self.lock:
            return self.flat.reference_vector().to("cpu")

    def _pack(self, grads: list, blocking: bool = False) -> list:
        """Copy received flat gradients into one aligned [n, ld] device buffer; return row views.

        ``blocking``: the sources are mailbox slots that RPC threads may rewrite as soon
        as this returns, so the host waits for the DMA."""
        n = len(grads)
        d = grads[0].numel()
        ld = padded(d)
        if self._gbuf is None or self._gbuf.shape[0] < n or self._gbuf.shape[1] != ld:
            self._gbuf = torch.zeros((max(n, self.num_workers), ld), dtype=torch.float32, device=self.device)
        for i, g in enumerate(grads):
            self._gbuf[i, :d].copy_(g, non_blocking=not blocking)
        return [self._gbuf[i, :d] for i in range(n)]

    def _mailbox(self, d: int):
        """Pinned C++ inbox with one slot per worker (created on first use)."""
        mb = getattr(self, "_mb", None)
        if mb is None or mb.slot_bytes < 4 * d:
            from garfield_amd import _native

            C = _native.native()
            mb = C.Mailbox(self.num_workers, 4 * d, self.device.type == "cuda")
            self._mb = mb
        return mb

    def get_gradients(self, iter_num, num_wait_wrk=-1):
        """Ask every worker for a gradient on the current model; return the first
        ``num_wait_wrk`` (default n - f) received, on the server's device.

        Replies land in the native pinned ``Mailbox`` (RPC threads copy into slot i
        without the GIL, tagged with the iteration); the server blocks in C++ until
        ``num_wait_wrk`` slots carry this iteration's tag, then DMAs exactly those
        slots into the aligned device buffer. Late replies of older iterations can
        never be mistaken for current ones (tag mismatch)."""
        if num_wait_wrk < 0:
            num_wait_wrk = self.num_workers - self.byz_wrk
        self.model.train()
        self.optimizer.zero_grad(set_to_none=False)
        payload = self._payload()
        d = self.flat.d
        try:
            mb = self._mailbox(d)
        except RuntimeError:
            mb = None  # native extension unavailable (CPU-only fallback)
        if mb is None:
            q = _Quorum(self.num_workers)
            for i, (rref, typ) in enumerate(zip(self.workers_rref, self.workers_types)):
                _remote_method_async(typ.compute_gradients, rref, iter_num, payload).then(q.callback(i, lambda r: r[1]))
            grads = q.wait(num_wait_wrk, self.rpc_timeout)
            self.build_graph(iter_num)
            return self._pack(grads)
        errors = []

        def make_cb(slot):
            def cb(fut):
                try:
                    mb.write(slot, iter_num, fut.wait()[1])
                except Exception as e:  # surface remote failures
                    errors.append(e)
                    mb.publish(slot, -2)
            return cb

        for i, (rref, typ) in enumerate(zip(self.workers_rref, self.workers_types)):
            _remote_method_async(typ.compute_gradients, rref, iter_num, payload).then(make_cb(i))
        self.build_graph(iter_num)   # overlaps the workers' computation
        timeout = -1.0 if self.rpc_timeout is None else float(self.rpc_timeout)
        slots = mb.wait(iter_num, num_wait_wrk, timeout)
        if len(slots) < num_wait_wrk:
            if errors:
                raise errors[0]
            raise TimeoutError(f"only {len(slots)} of {num_wait_wrk} gradients arrived for iteration {iter_num}")
        slots = slots[:num_wait_wrk]
        return self._pack([mb.tensor(i, d, torch.float32) for i in slots], blocking=True)

    def get_models(self, num_wait_ps=-1):
        if num_wait_ps < 0:
            num_wait_ps = self.num_ps - self.byz_ps
        q = _Quorum(self.num_ps)
        for i, (rref, typ) in enumerate(zip(self.ps_rref, self.ps_types)):
            _remote_method_async(typ.get_model, rref).then(q.callback(i, lambda r: r[1]))
        return [m.to(self.device) for m in q.wait(num_wait_ps, self.rpc_timeout)]

    def build_graph(self, iter_num):
        """Forward pass of the server model on one batch (updates BatchNorm statistics)."""
        data, _ = self.train_set[iter_num % len(self.train_set)]
        with self.lock, torch.no_grad():
            self.model(data)

    def get_model(self):
        return self.rank, self._payload()

    @property
    def latest_aggr_grad(self):
        return self._latest

    @latest_aggr_grad.setter
    def latest_aggr_grad(self, grad) -> None:
        """Assigning publishes the gradient to peers waiting in get_latest_aggr_grad."""
        with self.lock:
            self._latest = None if grad is None else grad.detach().clone()
        if grad is None:
            self._aggr_ready.clear()
        else:
            self._aggr_ready.set()

    def get_latest_aggr_grad(self):
        self._aggr_ready.wait()
        with self.lock:
            return self.rank, self._latest.to("cpu")

    def set_latest_aggr_grad(self, grad: torch.Tensor) -> None:
        self.latest_aggr_grad = grad

    def get_aggr_grads(self, num_wait_ps=-1):
        if num_wait_ps < 0:
            num_wait_ps = self.num_ps - self.byz_ps
        q = _Quorum(self.num_ps)
        for i, (rref, typ) in enumerate(zip(self.ps_rref, self.ps_types)):
            _remote_method_async(typ.get_latest_aggr_grad, rref).then(q.callback(i, lambda r: r[1]))
        return [g.to(self.device) for g in q.wait(num_wait_ps, self.rpc_timeout)]

    def _snapshot(self) -> nn.Module:
        with self.lock:
            return copy.deepcopy(self.model)

    @torch.no_grad()
    def compute_accuracy(self):
        m = self._snapshot()
        m.eval()
        correct = total = 0
        for x, y in self.test_set:
            pred = m(x).argmax(1)
            correct += int((pred == y).sum())
            total += y.numel()
        return correct * 100 / max(total, 1)

    @torch.no_grad()
    def compute_binary_accuracy(self):
        m = self._snapshot()
        m.eval()
        correct = total = 0
        for x, y in self.test_set:
            pred = m(x).round()
            correct += int((pred.view_as(y) == y).sum())
            total += y.numel()
        return correct * 100 / max(total, 1)

    def update_model(self, grad):
        """Apply a reference-layout flat gradient with the server's optimizer."""
        grad = grad.to(self.device, non_blocking=True)
        with self.lock:
            pos = 0
            for p in self.flat.params:
                n = p.numel()
                p.grad.copy_(grad[pos:pos + n].view(p.shape))
                pos += n
            self.optimizer.step()

    def write_model(self, model):
        """Replace the parameters by a reference-layout flat vector."""
        with self.lock:
            self.flat.load_reference_vector(model.to(self.device))

    # RPC benchmark helpers (reference server.py:300-305)
    def get_fake_models(self):
        futs = [_remote_method_async(typ.get_fake_model, rref) for rref, typ in zip(self.ps_rref, self.ps_types)]
        return [f.wait().to(self.device) for f in futs]

    def get_fake_model(self):
        m = getattr(self, "fake_model", None)
        return (m if m is not None else self.flat.reference_vector()).to("cpu")
