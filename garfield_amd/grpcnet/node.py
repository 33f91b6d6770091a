"""Nodes of the gRPC transport: ``Server`` (base), ``Worker``, ``PS``, ``ByzWorker``,
``ByzPS``.

Reference: ``tensorflow_impl/libs/{server,worker,ps,byz_worker,byz_ps}.py``. The
protocol is the reference's pull model: iteration ``t`` of a PS's model history is
the model *before* its t-th update (entry 0 = initial weights); a worker pulls
``GetModel(t)`` from every PS, aggregates them with the model rule, computes the
gradient of batch ``t`` of its partition and commits it as ``GetGradient(t)``; the
PS pulls those, aggregates with the gradient rule, applies its optimizer (Adam 1e-3,
``ps.py:56``) and commits model ``t+1``.

MI355X-first: models and GAR inputs stay on the GPU when one is present (the flat
vectors come off the wire into pinned host memory and are copied to the device
once); the GAR is the framework's HIP implementation; pulls from all peers are
concurrent and may stop at a quorum of the fastest replies. All nodes seed the model
initialisation identically, so every replica starts from the same weights.
"""
from __future__ import annotations

import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

from garfield_amd.data.datasets import DeviceLoader, fetch
from garfield_amd.grpcnet import service as svc
from garfield_amd.grpcnet.attacker import Attacker
from garfield_amd.models import NUM_CLASSES, build_model
from garfield_amd.models.nets import MLP
from garfield_amd.utils.flat import flat_parameters, write_flat_parameters

# TF model names (reference libs/model.py:48-58) → framework models
TF_MODELS = {"CNN": "cnn", "Cifarnet": "cifarnet", "MobileNetV2": "mobilenetv2", "Resnet50": "resnet50",
             "Resnet200": "resnet200", "VGG": "vgg16", "DenseNet": "densenet121", "Inception": "inception_v3"}


def build_tf_model(name: str, dataset: str) -> torch.nn.Module:
    classes = NUM_CLASSES.get(dataset, 10)
    if name.startswith("experiment:"):   # Garfield_legacy ``--experiment`` (apps/experiments.py)
        from garfield_amd.apps.experiments import instantiate

        return instantiate(name.split(":", 1)[1]).model()
    if name == "Small":   # Flatten → Dense(128, relu) → Dense(classes)
        sample = fetch(dataset, train=False).x[:1]
        return MLP(num_classes=classes, in_features=int(np.prod(sample.shape[1:])))
    return build_model(TF_MODELS.get(name, name), classes, dataset)


def training_progression(total: int, it: int, accuracy: float) -> None:
    """Reference ``libs/tools.py:162-165`` progress bar."""
    i = int(it / max(total - 1, 1) * 20)
    sys.stdout.write(f"\rTraining |{chr(0x2588) * i}{'.' * (20 - i)} | iter: {it}/{total - 1} "
                     f"Accuracy: {accuracy:.2f}%")
    sys.stdout.flush()


class Server:
    """Superclass of every gRPC node (reference ``libs/server.py:48-164``)."""

    job = "node"

    def __init__(self, network=None, log=False, dataset="mnist", model="Small", batch_size=128, nb_byz_worker=0,
                 device=None, keep: int = 64, seed: int = 1234, retries: int = 10, retry_delay: float = 5.0,
                 test_batch: int = 600, bind_host: str | None = None):
        self.log = log
        self.network = network
        self.nb_byz_worker = nb_byz_worker
        self.batch_size = batch_size
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.task_id = network.get_task_index()
        self.retries, self.retry_delay = retries, retry_delay
        self.dataset = dataset

        torch.manual_seed(seed)   # identical initial weights on every node
        self.model = build_tf_model(model, dataset).to(self.device)
        self._load_data(dataset, batch_size, test_batch, seed)

        self.ps_hosts = network.get_all_ps()
        self.worker_hosts = network.get_all_other_worker()
        self.ps_connections = [svc.Stub(h) for h in self.ps_hosts]
        self.worker_connections = [svc.Stub(h) for h in self.worker_hosts]
        self.port = int(network.get_my_port())

        self.service = svc.MessageExchangeService(self.flat_model(), keep=keep)
        self.server, self.bound_port = svc.make_server(self.service, self.port, host=bind_host)
        self.aggregated_weights = None

    # data -------------------------------------------------------------------------------
    def _partition(self, n_train: int):
        """PS: the whole train set; worker i of n: the i-th contiguous 1/n slice
        (reference ``libs/dataset.py:69-87``, percent split)."""
        if self.network.get_task_type() == "ps":
            return range(n_train)
        n = max(len(self.network.get_all_workers()), 1)
        size = n_train // n
        return range(self.task_id * size, min(n_train, (self.task_id + 1) * size))

    def _load_data(self, dataset, batch_size, test_batch, seed):
        train = fetch(dataset, train=True)
        test = fetch(dataset, train=False)
        self.train_data = DeviceLoader(train, self._partition(len(train)), batch_size, self.device, shuffle=True,
                                       seed=seed + self.task_id)
        self.test_data = DeviceLoader(test, range(len(test)), test_batch, self.device)

    # model ------------------------------------------------------------------------------
    def flat_model(self) -> torch.Tensor:
        return flat_parameters(self.model).detach()

    def write_model(self, model) -> None:
        if isinstance(model, np.ndarray):
            model = torch.from_numpy(model)
        write_flat_parameters(self.model, model.to(self.device, torch.float32))

    @torch.no_grad()
    def compute_accuracy(self) -> float:
        was = self.model.training
        self.model.eval()
        correct = total = 0
        for x, y in self.test_data:
            correct += int((self.model(x).argmax(1) == y).sum())
            total += int(y.numel())
        self.model.train(was)
        return 100.0 * correct / max(total, 1)

    # transport --------------------------------------------------------------------------
    def start(self) -> None:
        self.server.start()
        if self.log:
            print(f"Starting on port: {self.bound_port}", flush=True)

    def stop(self, grace: float | None = 1.0) -> None:
        self.server.stop(grace)
        for s in self.ps_connections + self.worker_connections:
            s.close()

    def wait_until_termination(self, timeout: float | None = None) -> None:
        self.server.wait_for_termination(timeout)

    def _to_device(self, replies) -> list[torch.Tensor]:
        out = []
        for _, arr in sorted(replies, key=lambda r: r[0]):   # deterministic GAR input order
            t = torch.from_numpy(arr.copy())
            if self.device.type == "cuda":
                t = t.pin_memory().to(self.device, non_blocking=True)
            out.append(t)
        return out

    def get_models(self, iter, quorum: int | None = None) -> list[torch.Tensor]:
        """Models of iteration ``iter`` from the PS replicas (fastest ``quorum``)."""
        replies = svc.pull(self.ps_connections, "GetModel", iter, self.job, self.task_id, quorum,
                           retries=self.retries, retry_delay=self.retry_delay)
        return self._to_device(replies)


class Worker(Server):
    """Computes gradients on its data partition (reference ``libs/worker.py:38-107``)."""

    job = "worker"

    def compute_gradients(self, iter):
        x, y = self.train_data[iter]
        self.model.train()
        for p in self.model.parameters():
            p.grad = None
        loss = F.cross_entropy(self.model(x), y)
        loss.backward()
        grad = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                          for p in self.model.parameters()])
        return float(loss.detach()), grad

    def commit_gradients(self, grads) -> None:
        self.service.gradients_history.append(grads)

    def linger(self, max_iter: int, timeout: float = 60.0) -> None:
        """Serve until every PS pulled the last gradient (the reference serves forever)."""
        self.service.wait_served("GetGradient", max_iter - 1, len(self.ps_hosts), timeout)


class PS(Server):
    """Parameter server (reference ``libs/ps.py:38-109``): Adam(1e-3) by default."""

    job = "ps"

    def __init__(self, *args, optimizer: str = "adam", lr: float = 1e-3, **kwargs):
        super().__init__(*args, **kwargs)
        params = list(self.model.parameters())
        if optimizer == "adam":
            self.optimizer = torch.optim.Adam(params, lr=lr)
        elif optimizer == "sgd":
            self.optimizer = torch.optim.SGD(params, lr=lr)
        elif optimizer == "rmsprop":
            self.optimizer = torch.optim.RMSprop(params, lr=lr)
        else:
            raise ValueError(f"unknown optimizer {optimizer!r}")

    def get_gradients(self, iter, quorum: int | None = None) -> list[torch.Tensor]:
        replies = svc.pull(self.worker_connections, "GetGradient", iter, self.job, self.task_id, quorum,
                           retries=self.retries, retry_delay=self.retry_delay)
        return self._to_device(replies)

    def update_model(self, gradient) -> torch.Tensor:
        if isinstance(gradient, np.ndarray):
            gradient = torch.from_numpy(gradient)
        g = gradient.to(self.device, torch.float32)
        off = 0
        for p in self.model.parameters():
            n = p.numel()
            p.grad = g[off:off + n].view_as(p).clone()
            off += n
        self.optimizer.step()
        return self.flat_model()

    upate_model = update_model   # the reference's spelling (ps.py:91)

    def commit_model(self, model) -> None:
        self.service.model_weights_history.append(model)

    def linger(self, max_iter: int, timeout: float = 60.0) -> None:
        """Serve until every worker and PS pulled the last model they need."""
        need = len(self.worker_hosts) + len(self.ps_hosts)
        self.service.wait_served("GetModel", max_iter - 1, need, timeout)


class ByzWorker(Worker):
    """Byzantine worker (reference ``libs/byz_worker.py:35-61``)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.attacker = Attacker(self.network.get_my_attack(), seed=1000 + self.task_id)

    def compute_gradients(self, iter, **kwargs):
        loss, gradient = super().compute_gradients(iter)
        est = None
        if self.attacker.needs_estimates:
            # colluders' honest estimates on the next batches (reference :55-57)
            est = [super(ByzWorker, self).compute_gradients(iter + 1 + i)[1]
                   for i in range(max(self.nb_byz_worker - 1, 0))]
        return loss, self.attacker.attack(gradient, est)


class ByzPS(PS):
    """Byzantine parameter server (reference ``libs/byz_ps.py:35-59``): commits an
    attacked model."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.attacker = Attacker(self.network.get_my_attack(), seed=2000 + self.task_id)

    def commit_model(self, model, **kwargs) -> None:
        self.service.model_weights_history.append(self.attacker.attack(model))
