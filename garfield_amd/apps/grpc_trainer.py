"""gRPC trainers: AggregaThor, ByzSGD and LEARN over the ``MessageExchange`` service.

Reference: ``tensorflow_impl/applications/{AggregaThor,ByzSGD,LEARN}/trainer.py``.

* ``--app aggregathor`` (``AggregaThor/trainer.py:55-97``): workers pull the PS
  models, aggregate them with the model rule, compute and commit gradients; the PS
  takes ``models[0]``, pulls the gradients, aggregates with the gradient rule,
  updates and commits.
* ``--app byzsgd`` (``ByzSGD/trainer.py:55-97``): as above, but every PS aggregates
  the models of all PS replicas with the model rule before its update.
* ``--app learn`` (``LEARN/trainer.py:51-90``): every process is a PS *and* a worker
  (``--config_ps`` / ``--config_w``).

Flags follow the reference (``--config --log --max_iter --dataset --model
--batch_size --nbbyzwrks --native``) plus ``--acc_freq`` (200 in the reference),
``--quorum_w`` / ``--quorum_ps`` (fastest-replies quorum; default: everyone),
``--device``, ``--lr``/``--optimizer`` and ``--linger`` (seconds a finished node keeps
serving its peers; the reference serves forever).
"""
from __future__ import annotations

import argparse
import json
import time

from garfield_amd.grpcnet.aggregator import Aggregator_tf
from garfield_amd.grpcnet.network import Network
from garfield_amd.grpcnet.node import PS, ByzPS, ByzWorker, Worker, training_progression


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--app", choices=["aggregathor", "byzsgd", "learn"], default="aggregathor")
    ap.add_argument("--config", default="TF_CONFIG")
    ap.add_argument("--config_w", default=None)
    ap.add_argument("--config_ps", default=None)
    ap.add_argument("--log", action="store_true")
    ap.add_argument("--max_iter", type=int, default=2000)
    ap.add_argument("--dataset", default="mnist")
    ap.add_argument("--model", default="Small")
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--nbbyzwrks", type=int, default=0)
    ap.add_argument("--native", action="store_true")
    ap.add_argument("--acc_freq", type=int, default=200)
    ap.add_argument("--quorum_w", type=int, default=-1)
    ap.add_argument("--quorum_ps", type=int, default=-1)
    ap.add_argument("--device", default=None)
    ap.add_argument("--optimizer", default="adam")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--linger", type=float, default=60.0)
    ap.add_argument("--retry_delay", type=float, default=5.0)
    ap.add_argument("--summary", default=None, help="write a JSON summary of the run here")
    return ap.parse_args(argv)


def _common(a):
    return dict(log=a.log, dataset=a.dataset, model=a.model, batch_size=a.batch_size, nb_byz_worker=a.nbbyzwrks,
                device=a.device, retry_delay=a.retry_delay)


def _q(v):
    return None if v is None or v < 0 else v


def run_worker(a, n: Network) -> dict:
    cls = ByzWorker if n.get_my_attack() != "None" else Worker
    w = cls(n, **_common(a))
    w.start()
    model_gar = Aggregator_tf(n.get_model_strategy(), len(n.get_all_ps()), 0, a.native)
    losses = []
    for it in range(a.max_iter):
        models = w.get_models(it, _q(a.quorum_ps))
        w.write_model(model_gar.aggregate(models))
        loss, grads = w.compute_gradients(it)
        w.commit_gradients(grads)
        losses.append(loss)
    w.linger(a.max_iter, a.linger)
    w.stop()
    return {"role": "worker", "index": n.get_task_index(), "losses": losses}


def run_ps(a, n: Network, aggregate_models: bool) -> dict:
    cls = ByzPS if n.get_my_attack() != "None" else PS
    p = cls(n, **_common(a), optimizer=a.optimizer, lr=a.lr)
    p.start()
    n_workers = len(n.get_all_workers())
    model_gar = Aggregator_tf(n.get_model_strategy(), len(n.get_all_ps()), 0, a.native)
    grad_gar = Aggregator_tf(n.get_gradient_strategy(), n_workers, a.nbbyzwrks, a.native)
    accuracy, accs = 0.0, []
    t0 = time.time()
    for it in range(a.max_iter):
        models = p.get_models(it, _q(a.quorum_ps))
        p.write_model(model_gar.aggregate(models) if aggregate_models else models[0])
        grads = p.get_gradients(it, _q(a.quorum_w))
        model = p.update_model(grad_gar.aggregate(grads))
        p.commit_model(model)
        if a.log:
            training_progression(a.max_iter, it, accuracy)
        if a.acc_freq > 0 and (it % a.acc_freq == 0 or it == a.max_iter - 1):
            accuracy = p.compute_accuracy()
            accs.append((it, accuracy))
    elapsed = time.time() - t0
    if a.log:
        print("\nTraining done!", flush=True)
    p.linger(a.max_iter, a.linger)
    p.stop()
    return {"role": "ps", "index": n.get_task_index(), "accuracy": accs, "seconds": elapsed}


def run_learn(a) -> dict:
    n_ps, n_w = Network(a.config_ps), Network(a.config_w)
    p = (ByzPS if n_ps.get_my_attack() != "None" else PS)(n_ps, **_common(a), optimizer=a.optimizer, lr=a.lr)
    w = (ByzWorker if n_w.get_my_attack() != "None" else Worker)(n_w, **_common(a))
    p.start()
    w.start()
    model_gar = Aggregator_tf(n_ps.get_model_strategy(), len(n_w.get_all_ps()), a.nbbyzwrks, a.native)
    grad_gar = Aggregator_tf(n_ps.get_gradient_strategy(), len(n_ps.get_all_workers()), a.nbbyzwrks, a.native)
    accuracy, accs, losses = 0.0, [], []
    for it in range(a.max_iter):
        agg = model_gar.aggregate(w.get_models(it, _q(a.quorum_ps)))
        w.write_model(agg)
        p.write_model(agg)
        loss, grads = w.compute_gradients(it)
        w.commit_gradients(grads)
        losses.append(loss)
        model = p.update_model(grad_gar.aggregate(p.get_gradients(it, _q(a.quorum_w))))
        p.commit_model(model)
        if a.log:
            training_progression(a.max_iter, it, accuracy)
        if a.acc_freq > 0 and (it % a.acc_freq == 0 or it == a.max_iter - 1):
            accuracy = p.compute_accuracy()
            accs.append((it, accuracy))
    p.linger(a.max_iter, a.linger)
    w.linger(a.max_iter, a.linger)
    p.stop()
    w.stop()
    return {"role": "learn", "index": n_ps.get_task_index(), "accuracy": accs, "losses": losses}


def main(argv=None):
    a = parse_args(argv)
    if a.app == "learn":
        out = run_learn(a)
    else:
        n = Network(a.config)
        if n.get_task_type() == "worker":
            out = run_worker(a, n)
        elif n.get_task_type() == "ps":
            out = run_ps(a, n, aggregate_models=a.app == "byzsgd")
        else:
            raise SystemExit("Unknown task type, please check TF_CONFIG file")
    if a.summary:
        with open(a.summary, "w") as fh:
            json.dump(out, fh)
    return out


if __name__ == "__main__":
    main()
