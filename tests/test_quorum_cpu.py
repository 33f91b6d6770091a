"""Fastest-quorum aggregation on collectives (parallel/quorum.py), 3 gloo ranks on CPU.

Reference semantics: the PS aggregates the fastest n - f gradients
(pytorch_impl/libs/garfieldpp/server.py:134-155)."""
import os
import socket
import tempfile
import time

import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.parallel.quorum import QuorumConfig, QuorumDataParallel
from garfield_amd.parallel.engine import synthetic_batches


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


STEPS, DELAY = 6, 1.0


def _worker(rank, world, port, outdir, quorum, delay, byz=None, gar="median", sync=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from garfield_amd.parallel.comm import init_distributed, shutdown

    ctx = init_distributed(backend="gloo", device="cpu")
    torch.manual_seed(0)
    byz = {1: "reverse"} if byz is None else byz
    if sync:   # the synchronous engine, for comparison
        from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel

        eng = RobustDataParallel(build_model("mlp"), F.nll_loss, ctx,
                                 EngineConfig(gar=gar, f=1, workers_per_rank=2, lr=0.05, byzantine=byz,
                                              shard_gar=False, collusion="all"))
        eng.last_quorum, eng.skipped, eng.finish = None, 0, (lambda: None)
    else:
        eng = QuorumDataParallel(build_model("mlp"), F.nll_loss, ctx,
                                 QuorumConfig(gar=gar, f=1, workers_per_rank=2, quorum=quorum, lr=0.05,
                                              byzantine=byz, straggler_delay={2: delay}, collusion="all"))
    b = synthetic_batches(2, 8, (1, 28, 28), 10, "cpu", seed=rank)
    eng.step(b)   # warm-up (process groups connect)
    t0 = time.time()
    quorums = []
    for _ in range(STEPS):
        eng.step(b)
        quorums.append(eng.last_quorum)
    elapsed = time.time() - t0
    eng.finish()
    torch.save({"flat": eng.flat_model().clone(), "t": elapsed, "q": quorums, "skipped": eng.skipped, "w": eng.last_weights},
               os.path.join(outdir, f"r{rank}.pt"))
    shutdown(ctx)


def _run(quorum, delay, *extra):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(3, free_port(), d, quorum, delay, *extra), nprocs=3, join=True)
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(3)]


def test_straggler_outside_the_quorum_does_not_slow_the_others():
    out = _run(quorum=2, delay=DELAY)
    # every replica applied the same updates (the leader's quorum sets, the same rows)
    assert torch.equal(out[0]["flat"], out[1]["flat"]) and torch.equal(out[0]["flat"], out[2]["flat"])
    # ranks 0 / 1 never waited for rank 2's delayed rows
    assert all(q == [0, 1] for q in out[0]["q"])
    # (waiting would take >= STEPS * DELAY; the margin absorbs a loaded CI host)
    assert out[0]["t"] < 0.6 * STEPS * DELAY, out[0]["t"]
    assert out[1]["t"] < 0.6 * STEPS * DELAY, out[1]["t"]
    assert torch.isfinite(out[0]["flat"]).all()


def test_full_quorum_waits_for_everyone_and_matches():
    out = _run(quorum=3, delay=0.2)
    assert all(q == [0, 1, 2] for q in out[0]["q"])
    assert out[0]["t"] >= STEPS * 0.2 * 0.9
    assert torch.equal(out[0]["flat"], out[2]["flat"])


def test_colluding_attacker_with_straggler_keeps_replicas_identical():
    """A lie (colluding) slot + a straggler outside the quorum: the attack runs on a copy of
    the chosen rows, so the straggler, which receives the rows late, attacks the same
    honest rows and every replica applies the same update."""
    out = _run(2, 0.5, {1: "lie", 4: "empire"})
    assert torch.equal(out[0]["flat"], out[1]["flat"]) and torch.equal(out[0]["flat"], out[2]["flat"])


def test_full_quorum_equals_the_synchronous_engine():
    """Quorum rows in slot order (j * world + r): with every rank in the quorum, Krum picks
    and weighs exactly what the synchronous engine does."""
    q = _run(3, 0.0, {1: "reverse"}, "krum")
    s = _run(3, 0.0, {1: "reverse"}, "krum", True)
    assert torch.equal(q[0]["flat"], s[0]["flat"])
