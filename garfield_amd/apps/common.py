"""Shared CLI / launch helpers of the applications.

The flags are the reference trainers' (``applications/*/trainer.py``: ``--master
--rank --dataset --batch --num_ps --num_workers --fw --fps --model --loss
--optimizer --opt_args --num_iter --gar --acc_freq --bench --log``; LEARN:
``--num_nodes --f --non_iid``); ``--bench`` / ``--log`` accept true/false strings
(the reference's ``type=bool`` treated any non-empty string as True).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

from garfield_amd.utils.logging import info


def str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).lower() in ("1", "true", "yes", "y", "on")


def add_common(p: argparse.ArgumentParser, ps: bool = True) -> argparse.ArgumentParser:
    p.add_argument("--master", type=str, default="127.0.0.1", help="Master node (rank 0) address.")
    p.add_argument("--port", type=int, default=29500, help="Rendezvous port (MASTER_PORT).")
    p.add_argument("--rank", type=int, default=0, help="Rank of this process.")
    p.add_argument("--dataset", type=str, default="mnist", help="mnist, cifar10, pima, synthetic, ...")
    p.add_argument("--batch", type=int, default=32, help="Minibatch size of each worker.")
    if ps:
        p.add_argument("--num_ps", type=int, default=1, help="Number of parameter servers.")
        p.add_argument("--num_workers", type=int, default=1, help="Number of workers.")
        p.add_argument("--fw", type=int, default=0, help="Number of declared Byzantine workers.")
        p.add_argument("--fps", type=int, default=0, help="Number of declared Byzantine servers.")
    p.add_argument("--model", type=str, default="convnet")
    p.add_argument("--loss", type=str, default="nll")
    p.add_argument("--optimizer", type=str, default="sgd")
    p.add_argument("--opt_args", type=json.loads, default={"lr": "0.1"},
                   help='Optimizer arguments as JSON, e.g. \'{"lr":"0.1"}\'')
    p.add_argument("--num_iter", type=int, default=5000)
    p.add_argument("--gar", type=str, default="average")
    p.add_argument("--acc_freq", type=int, default=100, help="Accuracy evaluation period (iterations).")
    p.add_argument("--bench", type=str2bool, default=False, help="Print per-step timing and bandwidth.")
    p.add_argument("--log", type=str2bool, default=False, help="Print the loss at each iteration.")
    p.add_argument("--attack", type=str, default="",
                   help="Attack of the declared Byzantine nodes (random|reverse|drop|lie|empire); empty = honest.")
    p.add_argument("--train_size", type=int, default=None)
    p.add_argument("--device", type=str, default=None, help="cpu / cuda (default: cuda when available)")
    p.add_argument("--rpc_timeout", type=float, default=600.0)
    return p


def print_setup(rank: int, **fields) -> None:
    info(f"**** SETUP AT NODE {rank} ***")
    for k, v in fields.items():
        info(f"{k}: {v}")
    info("------------------------------------")
    sys.stdout.flush()


def init_rpc(name: str, rank: int, world_size: int, master: str, port: int, timeout: float = 600.0,
             num_threads: int = 16) -> None:
    import torch.distributed.rpc as rpc

    os.environ["MASTER_ADDR"] = master
    os.environ["MASTER_PORT"] = str(port)
    opts = rpc.TensorPipeRpcBackendOptions(num_worker_threads=num_threads, rpc_timeout=timeout,
                                           init_method=f"tcp://{master}:{port}")
    rpc.init_rpc(name, rank=rank, world_size=world_size, rpc_backend_options=opts)


def seed_all(seed: int = 1234) -> None:
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


class StepTimer:
    """``--bench`` support: wall time and NIC bytes of one training step."""

    def __init__(self, enabled: bool):
        self.enabled = enabled

    def __enter__(self):
        if self.enabled:
            from garfield_amd.runtime.tools import get_bytes_com

            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self.t0 = time.perf_counter()
            self.b0 = get_bytes_com()
        return self

    def __exit__(self, *exc):
        if self.enabled:
            from garfield_amd.runtime.tools import convert_to_gbit, get_bytes_com

            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self.seconds = time.perf_counter() - self.t0
            self.gbit = convert_to_gbit(get_bytes_com() - self.b0)
        return False
