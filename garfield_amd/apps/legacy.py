"""Garfield_legacy: the original Byzantine-resilient PS protocol (TF1 system) over gRPC.

Reference: ``tensorflow_impl/applications/Garfield_legacy/byzPS.py`` and
``byzWorker.py`` (flags ``--vanilla / --asyncr / --smart``, ``--nbbyzwrk``,
``--nbbyzps``, ``--less_grad``, ``--rate``, ``--l``, ``--max_steps``,
``--eval_steps``), ``experiments/mnistAttack.py`` (malformed inputs). Unlike the
TF2 applications, workers keep their own model replica and apply the
*aggregated gradients* the parameter servers publish. Iteration t:

worker
  * t > 0: pull the PSes' aggregated gradient of iteration t and apply it with
    RMSProp(rate): ``--vanilla`` one PS (PS 0); ``--asyncr`` the fastest
    2·f_ps + 3 PSes, aggregated with Krum (the median when no Byzantine PS is
    declared: Krum needs f >= 1); ``--smart`` one PS (round robin), all PSes
    aggregated the same way every T = 1 / (3 l rate) iterations;
  * compute the gradient of batch t on the new model and publish it;
  * ``--smart``: Kardam Lipschitz filter (``runtime/kardam.py``).
PS
  * t > 0: publish the aggregate of iteration t - 1 as the aggregated gradient t;
  * pull the worker gradients of iteration t (all; 2·f_w + 3 with ``--asyncr`` or
    ``--less_grad``), aggregate with Krum (Average for ``--vanilla``);
  * ``--asyncr``, or ``--smart`` at multiples of T: exchange the aggregates among
    the PSes (fastest 2·f_ps + 3, or all), take their median, apply it; otherwise
    apply the aggregate itself.

Nodes talk over the reference's legacy ``TrainMessageExchange`` service
(``all.proto``; ``grpcnet/service.py:TrainMessageExchangeService``): a PS publishes
its aggregated gradients in its gradient history (``GetGradients(iter)``) and uses
its model history for the PS-to-PS exchange (``GetModel``: entry t + 1 = aggregate of
iteration t; entry 0 is the initial model that workers pull first with
``GetUnifiedModel``); workers serve their gradients with ``GetGradients`` (plus the
Kardam Lipschitz value in ``--smart`` mode). Byzantine workers use the TF_CONFIG
attack (``Poison1``/``Poison2`` = the malformed-input attack of ``mnistAttack``);
a Byzantine PS corrupts the aggregate it publishes.
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from garfield_amd.data.datasets import poison_batch
from garfield_amd.grpcnet import service as svc
from garfield_amd.grpcnet.aggregator import Aggregator_tf
from garfield_amd.grpcnet.attacker import Attacker
from garfield_amd.grpcnet.network import Network
from garfield_amd.grpcnet.node import Server, Worker
from garfield_amd.runtime.kardam import LipschitzFilter
from garfield_amd.utils.flat import flat_parameters

POISON = {"Poison1": 1, "Poison2": 2}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--config", default="TF_CONFIG")
    mode = ap.add_mutually_exclusive_group()
    mode.add_argument("--vanilla", action="store_true", help="non-Byzantine baseline (Average, one PS)")
    mode.add_argument("--asyncr", action="store_true", help="quorums of 2f+3 and a PS median exchange every step")
    mode.add_argument("--smart", action="store_true", help="PS exchange every T steps + Lipschitz filter")
    ap.add_argument("--nbbyzwrk", type=int, default=0)
    ap.add_argument("--nbbyzps", type=int, default=0)
    ap.add_argument("--less_grad", action="store_true", help="PS collects only 2f+3 worker gradients")
    ap.add_argument("--rate", type=float, default=1e-3)
    ap.add_argument("--l", type=float, default=1.0, help="Lipschitz constant used for T = 1/(3 l rate)")
    ap.add_argument("--T", type=int, default=0, help="override the smart exchange period")
    ap.add_argument("--max_steps", type=int, default=1000)
    ap.add_argument("--eval_steps", type=int, default=100)
    ap.add_argument("--dataset", default="mnist")
    ap.add_argument("--model", default="Small")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--device", default=None)
    ap.add_argument("--log", action="store_true")
    ap.add_argument("--linger", type=float, default=60.0)
    ap.add_argument("--retry_delay", type=float, default=5.0)
    ap.add_argument("--summary", default=None)
    ap.add_argument("--experiment", default=None,
                    help="experiments registry name (mnist, mnistAttack, cnnet, slim-<model>-<dataset>, "
                         "byzPS.py:120); overrides --dataset / --model")
    a = ap.parse_args(argv)
    if a.experiment:
        from garfield_amd.apps.experiments import instantiate

        a.dataset = instantiate(a.experiment, [f"batch-size:{a.batch}"]).dataset
        a.model = f"experiment:{a.experiment}"
    return a


def period(a) -> int:
    return a.T if a.T > 0 else max(int(1.0 / (3.0 * a.l * a.rate)), 1)


def _optimizer(model, rate):
    return torch.optim.RMSprop(model.parameters(), lr=rate)


def _apply(node, opt, grad: torch.Tensor) -> None:
    g = grad.to(node.device, torch.float32)
    off = 0
    for p in node.model.parameters():
        n = p.numel()
        p.grad = g[off:off + n].view_as(p).clone()
        off += n
    opt.step()


def _quorum(n: int, f: int) -> int:
    return min(2 * f + 3, n)


def _use_legacy_service(node) -> None:
    """Talk to the peers over ``TrainMessageExchange`` (the reference's legacy service,
    ``all.proto``); every node serves it next to ``MessageExchange``."""
    for st in node.ps_connections + node.worker_connections:
        st.close()
    node.ps_connections = [svc.LegacyStub(h) for h in node.ps_hosts]
    node.worker_connections = [svc.LegacyStub(h) for h in node.worker_hosts]


class LegacyWorker(Worker):
    """Worker with its own replica (reference ``byzWorker.py``)."""

    def __init__(self, network, a):
        super().__init__(network, log=a.log, dataset=a.dataset, model=a.model, batch_size=a.batch,
                         nb_byz_worker=a.nbbyzwrk, device=a.device, retry_delay=a.retry_delay)
        self.a = a
        self.opt = _optimizer(self.model, a.rate)
        attack = network.get_my_attack()
        self.poison = POISON.get(attack, 0)
        self.attacker = Attacker(attack, seed=1000 + self.task_id) if attack not in ("None", *POISON) else None
        self._gen = torch.Generator().manual_seed(3000 + self.task_id)
        _use_legacy_service(self)

    def compute_gradients(self, iter):
        if not self.poison:
            loss, g = super().compute_gradients(iter)
        else:
            x, y = poison_batch(*self.train_data[iter], self.poison, self._gen)
            self.model.train()
            for p in self.model.parameters():
                p.grad = None
            out = torch.nn.functional.cross_entropy(self.model(x), y)
            out.backward()
            g = torch.cat([p.grad.reshape(-1) for p in self.model.parameters()])
            loss = float(out.detach())
        if self.attacker is not None:
            g = self.attacker.attack(g)
        return loss, g

    def pull_aggregates(self, it: int, ps_index: int | None, quorum: int | None) -> list[torch.Tensor]:
        stubs = self.ps_connections if ps_index is None else [self.ps_connections[ps_index]]
        replies = svc.pull(stubs, "GetGradients", it, self.job, self.task_id, quorum, retries=self.retries,
                           retry_delay=self.retry_delay)
        return self._to_device(replies)

    def unified_model(self) -> torch.Tensor:
        """The initial model from PS 0 (``GetUnifiedModel``)."""
        replies = svc.pull(self.ps_connections[:1], "GetUnifiedModel", 0, self.job, self.task_id, 1,
                           retries=self.retries, retry_delay=self.retry_delay)
        return self._to_device(replies)[0]


class LegacyPS(Server):
    """Parameter server (reference ``byzPS.py``)."""

    job = "ps"

    def __init__(self, network, a):
        super().__init__(network, log=a.log, dataset=a.dataset, model=a.model, batch_size=a.batch,
                         nb_byz_worker=a.nbbyzwrk, device=a.device, retry_delay=a.retry_delay)
        self.opt = _optimizer(self.model, a.rate)
        attack = network.get_my_attack()
        self.attacker = Attacker(attack, seed=2000 + self.task_id) if attack != "None" else None
        _use_legacy_service(self)

    def publish(self, it: int, aggregate: torch.Tensor) -> None:
        out = self.attacker.attack(aggregate) if self.attacker is not None else aggregate
        self.service.gradients_history.put(it, out)

    def worker_gradients(self, it: int, quorum: int | None) -> list[torch.Tensor]:
        replies = svc.pull(self.worker_connections, "GetGradients", it, self.job, self.task_id, quorum,
                           retries=self.retries, retry_delay=self.retry_delay)
        return self._to_device(replies)

    def exchange(self, it: int, aggregate: torch.Tensor, quorum: int | None) -> list[torch.Tensor]:
        self.service.model_weights_history.put(it + 1, aggregate)
        replies = svc.pull(self.ps_connections, "GetModel", it + 1, self.job, self.task_id, quorum,
                           retries=self.retries, retry_delay=self.retry_delay)
        return self._to_device(replies)


def run_worker(a, n: Network) -> dict:
    w = LegacyWorker(n, a)
    w.start()
    num_ps = len(n.get_all_ps())
    T = period(a)
    w.write_model(w.unified_model() if num_ps else w.flat_model())
    q_ps = _quorum(num_ps, a.nbbyzps) if a.asyncr else num_ps
    # the reference aggregates the PS replies with Krum(f_ps); Krum needs f >= 1 and
    # n >= 2f + 3, so without declared Byzantine PSes (or too few PSes) the median
    krum_ok = a.nbbyzps >= 1 and q_ps >= 2 * a.nbbyzps + 3
    krum_ps = Aggregator_tf("Krum" if krum_ok else "Median", q_ps, a.nbbyzps)
    kardam = LipschitzFilter(num_ps, a.nbbyzps) if a.smart else None
    losses, lip = [], []
    next_ps = 0
    for it in range(a.max_steps):
        if it > 0:
            if a.asyncr:
                up = krum_ps.aggregate(w.pull_aggregates(it, None, q_ps))
            elif a.smart and it % T == 0:
                up = krum_ps.aggregate(w.pull_aggregates(it, None, None))
            else:
                if a.smart:
                    next_ps = (next_ps + 1) % num_ps
                up = w.pull_aggregates(it, 0 if a.vanilla or not a.smart else next_ps, None)[0]
            _apply(w, w.opt, torch.as_tensor(up))
        loss, grad = w.compute_gradients(it)
        if kardam is not None:
            st = kardam.observe(grad, flat_parameters(w.model),
                                {"T": T, "iteration": it, "num_byz_workers": a.nbbyzwrk, "lr": a.rate,
                                 "num_workers": len(n.get_all_workers())})
            if st is not None:
                lip.append((it, st.lipschitz, st.threshold, st.accept))
                w.service.legacy.lipschitz[it] = float(st.lipschitz)   # served with GetGradients(it)
        w.commit_gradients(grad)
        losses.append(loss)
    w.linger(a.max_steps, a.linger)
    w.stop()
    out = {"role": "worker", "index": n.get_task_index(), "losses": losses}
    if kardam is not None:
        out["kardam"] = {"observed": kardam.observed, "rejected": kardam.rejected, "last": lip[-5:]}
    return out


def run_ps(a, n: Network) -> dict:
    p = LegacyPS(n, a)
    p.start()
    n_w, num_ps = len(n.get_all_workers()), len(n.get_all_ps())
    T = period(a)
    q_w = _quorum(n_w, a.nbbyzwrk) if (a.asyncr or a.less_grad) else None
    gar = Aggregator_tf("Average" if a.vanilla else "Krum", q_w or n_w, a.nbbyzwrk)
    med = Aggregator_tf("Median", num_ps, a.nbbyzps)
    q_ps = _quorum(num_ps, a.nbbyzps) if a.asyncr else None
    aggr, accs, last_exchange = None, [], None
    t0 = time.time()
    for it in range(a.max_steps):
        if it > 0:
            p.publish(it, aggr)
        grads = p.worker_gradients(it, q_w)
        aggr = torch.as_tensor(gar.aggregate(grads)).to(p.device, torch.float32)
        if a.asyncr or (a.smart and it % T == 0 and it > 0):
            aggr = torch.as_tensor(med.aggregate(p.exchange(it, aggr, q_ps))).to(p.device, torch.float32)
            last_exchange = it
        _apply(p, p.opt, aggr)
        if a.eval_steps > 0 and (it % a.eval_steps == 0 or it == a.max_steps - 1):
            accs.append((it, p.compute_accuracy()))
            if a.log:
                print(f"[PS {p.task_id}] iteration {it} accuracy {accs[-1][1]:.2f} "
                      f"elapsed {time.time() - t0:.1f}s", flush=True)
    elapsed = time.time() - t0
    # keep serving while peers may still need this PS (the reference sleeps 10 s):
    if q_w is not None and q_w < n_w:   # quorum pulls: wait for every worker's last gradient
        p.worker_gradients(a.max_steps - 1, None)   # (committed after its last pull of this PS)
    if last_exchange is not None:   # the other PSes' last exchange pulls
        p.service.wait_served("GetModel", last_exchange + 1, q_ps or num_ps, a.linger)
    p.stop()
    return {"role": "ps", "index": n.get_task_index(), "accuracy": accs, "seconds": elapsed}


def main(argv=None):
    a = parse_args(argv)
    if not (a.vanilla or a.asyncr or a.smart):
        a.vanilla = True
    n = Network(a.config)
    if n.get_task_type() == "worker":
        out = run_worker(a, n)
    elif n.get_task_type() == "ps":
        out = run_ps(a, n)
    else:
        raise SystemExit("Unknown task type, please check TF_CONFIG file")
    if a.summary:
        with open(a.summary, "w") as fh:
            json.dump(out, fh)
    return out


if __name__ == "__main__":
    main()
