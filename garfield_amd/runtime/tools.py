"""Factories and RPC glue of the node runtime (reference ``garfieldpp/tools.py:47-193``).

* ``select_loss`` / ``select_model`` / ``select_optimizer`` keep the reference names;
  models come from ``garfield_amd.models`` (torchvision architectures implemented
  in-tree) and are NOT wrapped in ``nn.DataParallel`` (one process per GPU here);
* ``_call_method`` / ``_remote_method_sync`` / ``_remote_method_async`` are the RPC
  helpers of the reference;
* ``get_server`` / ``get_worker`` wait on a ``threading.Event`` set when the local
  singleton registers, instead of the reference's sleep-poll loop.
"""
from __future__ import annotations

import threading

import psutil
import torch
import torch.nn as nn

from garfield_amd.models import NUM_CLASSES, build_model

server_instance = None
worker_instance = None
_server_ready = threading.Event()
_worker_ready = threading.Event()


def select_loss(loss_fn: str):
    losses = {"nll": nn.NLLLoss, "cross-entropy": nn.CrossEntropyLoss, "binary-cross-entropy": nn.BCELoss,
              "mse": nn.MSELoss}
    if loss_fn not in losses:
        raise ValueError(f"The selected loss function is undefined, available losses are: {list(losses)}")
    return losses[loss_fn]()


def select_model(model: str, device, dataset: str = "mnist") -> nn.Module:
    num_classes = NUM_CLASSES.get(dataset, 10)
    return build_model(model, num_classes=num_classes).to(device)


def select_optimizer(model: nn.Module, optimizer: str, *args, **kwargs):
    kwargs = {k: float(v) if isinstance(v, str) else v for k, v in kwargs.items()}  # --opt_args are JSON strings
    opts = {"sgd": torch.optim.SGD, "adam": torch.optim.Adam, "adamw": torch.optim.AdamW,
            "rmsprop": torch.optim.RMSprop, "adagrad": torch.optim.Adagrad}
    if optimizer not in opts:
        raise ValueError(f"The selected optimizer is undefined, available optimizers are: {list(opts)}")
    return opts[optimizer](model.parameters(), *args, **kwargs)


def adjust_learning_rate(optimizer, lr: float) -> None:
    for g in optimizer.param_groups:
        g["lr"] = lr


# ---------------------------------------------------------------------- RPC


def _call_method(method, rref, *args, **kwargs):
    """Call ``method`` on the object owned by ``rref`` (runs on the owner)."""
    return method(rref.local_value(), *args, **kwargs)


def _type_of(rref):
    """Class of the object owned by ``rref`` (runs on the owner; classes pickle by name)."""
    return type(rref.local_value())


def _remote_method_sync(method, rref, *args, **kwargs):
    from torch.distributed.rpc import rpc_sync

    return rpc_sync(rref.owner(), _call_method, args=[method, rref] + list(args), kwargs=kwargs)


def _remote_method_async(method, rref, *args, **kwargs):
    from torch.distributed.rpc import rpc_async

    return rpc_async(rref.owner(), _call_method, args=[method, rref] + list(args), kwargs=kwargs)


def register_server(s) -> None:
    global server_instance
    server_instance = s
    _server_ready.set()


def register_worker(w) -> None:
    global worker_instance
    worker_instance = w
    _worker_ready.set()


def get_server():
    _server_ready.wait()
    return server_instance


def get_worker():
    _worker_ready.wait()
    return worker_instance


# ---------------------------------------------------------------------- network accounting


def get_bytes_com() -> int:
    """Bytes sent + received on all NICs so far (reference tools.py:152-156)."""
    c = psutil.net_io_counters()
    return c.bytes_sent + c.bytes_recv


def convert_to_gbit(value: float) -> float:
    return value / 1024.0 / 1024.0 / 1024.0 * 8
