"""Worker node (reference ``garfieldpp/worker.py:52-96``).

``Worker(rank, world_size, num_workers, batch_size, model, dataset, loss, train_size=None)``
and ``compute_gradients(iter_num, model) -> (rank, flat_grad_cpu, loss)`` keep the
reference contract. MI355X-side differences:

* the training partition lives on the device (``DeviceLoader``) and batch
  ``iter_num % len(train_set)`` is produced there (fresh augmentation per epoch);
* the model a server sends is loaded into a device-resident replica
  (``load_state``: flat vector or ``nn.Module``), instead of moving the whole
  module to the GPU on every call (reference ``worker.py:86``);
* the gradient is flattened by the fused multi-tensor HIP kernel and copied to a
  pinned host buffer with one DMA.
"""
from __future__ import annotations

import logging
import threading

import torch
import torch.nn as nn

from garfield_amd.data.datasets import DatasetManager
from garfield_amd.runtime import tools
from garfield_amd.utils.flat import FlatParams

logger = logging.getLogger(__name__)


class Worker:
    """Byzantine-resilient worker (honest)."""

    def __init__(self, rank, world_size, num_workers, batch_size, model, dataset, loss, train_size=None,
                 device=None, register: bool = True):
        self.device = torch.device(device) if device else (
            torch.device("cuda") if torch.cuda.device_count() > 0 else torch.device("cpu"))
        self.rank = rank
        self.batch_size = batch_size
        self.loss = tools.select_loss(loss)
        self.model_name, self.dataset = model, dataset
        manager = DatasetManager(dataset, batch_size, num_workers, world_size, rank, train_size, device=self.device)
        self.train_set = manager.get_train_set()
        self.num_train_samples = len(self.train_set)
        self._replica: nn.Module | None = None
        self._flat: FlatParams | None = None
        self._host = None
        self._lock = threading.Lock()  # RPC handlers may call concurrently (e.g. LEARN: n servers)
        if register:
            tools.register_worker(self)

    # ------------------------------------------------------------------ #

    def _ensure_replica(self, model) -> nn.Module:
        if self._replica is None:
            if isinstance(model, nn.Module):
                import copy

                self._replica = copy.deepcopy(model).to(self.device)
            else:
                self._replica = tools.select_model(self.model_name, self.device, self.dataset)
            self._flat = FlatParams(self._replica, device=self.device, with_grad=False)
        return self._replica

    def load_state(self, model) -> None:
        """Load a server's model (``nn.Module`` or reference-layout flat vector)."""
        rep = self._ensure_replica(model)
        with torch.no_grad():
            if isinstance(model, nn.Module):
                for p, q in zip(rep.parameters(), model.parameters()):
                    p.copy_(q.detach(), non_blocking=True)
                for b, c in zip(rep.buffers(), model.buffers()):
                    b.copy_(c.detach(), non_blocking=True)
            else:
                self._flat.load_reference_vector(model.to(self.device, non_blocking=True))

    def flat_gradient(self) -> torch.Tensor:
        """Reference-layout flat fp32 gradient of the replica (device)."""
        return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                          for p in self._flat.params])

    def compute_local_gradient(self, iter_num: int, model=None):
        """Gradient on batch ``iter_num % len(train_set)``; returns (device flat grad, loss tensor)."""
        if model is not None:
            self.load_state(model)
        rep = self._replica
        rep.train()
        for p in self._flat.params:
            p.grad = None
        data, target = self.train_set[iter_num % self.num_train_samples]
        out = rep(data)
        loss = self.loss(out, target)
        loss.backward()
        return self.flat_gradient(), loss.detach()

    def compute_gradients(self, iter_num, model):
        """Reference contract: (rank, flat fp32 CPU gradient, loss float)."""
        with self._lock:
            grad, loss = self.compute_local_gradient(iter_num, model)
            if self._host is None or self._host.numel() != grad.numel():
                self._host = torch.empty(grad.numel(), dtype=torch.float32,
                                         pin_memory=self.device.type == "cuda")
            self._host.copy_(grad, non_blocking=True)
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            return self.rank, self._host.clone(), float(loss)
