"""Overlap of the bucketed exchange with the backward, measured WITHOUT a profiler
(rocprofv3's kernel trace serialises graph launches, so a traced run cannot show it).

Runs the bench configuration with ``--shard-gar`` on one GPU and the loopback exchange
(GARFIELD_LOOPBACK_EXCHANGE=1: each bucket is copied on the comm stream as the
all-to-all would move it), and reads HIP timing events: the step start, the end of the
grouped forward/backward graph (main stream) and the moment each bucket's exchange
finished on the comm stream. A bucket whose exchange finished before the graph ended
ran under the backward. With the forward staged at the bucket boundaries (the default
with a comm stream), it also reports when the previous step's layer3 / layer4+fc updates
ended relative to this step's forward start: positive = they ran beside the forward.

    GARFIELD_OVERLAP=1 python scripts/overlap_timing.py [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

os.environ.setdefault("GARFIELD_LOOPBACK_EXCHANGE", "1")
os.environ.setdefault("GARFIELD_EXCHANGE_TIMING", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from garfield_amd.data.fresh import DeviceBatches  # noqa: E402
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--plain", action="store_true", help="the unsharded engine (no buckets), for comparison")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if os.environ.get("DUMMY_STREAM"):
        _dummy = torch.cuda.Stream(dev)  # noqa: F841
    torch.manual_seed(1234)
    eng = RobustDataParallel(build_model(a.model, num_classes=10), F.cross_entropy, DistContext(device=dev),
                             EngineConfig(gar="krum", f=2, workers_per_rank=8, lr=0.01, cuda_graph=True,
                                          shard_gar=not a.plain))
    feed = DeviceBatches.synthetic(50000, (3, 32, 32), 10, 8, 250, dev, seed=1000)
    feed.attach(eng.grouped_inputs(250, (3, 32, 32)))
    marks = {}
    inner = eng._grouped_compute

    def timed_compute():
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        # the previous step's buckets still in flight on the comm stream (staged forward)
        marks["prev_ready"] = list(eng._shard._ready) if eng._shard is not None else []
        s0.record()
        inner()
        s1.record()
        marks["start"], marks["graph_end"] = s0, s1

    eng._grouped_compute = timed_compute
    for _ in range(4):
        eng.step(feed.next())
    torch.cuda.synchronize()
    # a.steps steps back to back (no host sync in between, as in training), events kept per step
    rounds = []
    for _ in range(a.steps):
        eng.step(feed.next())
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        rounds.append((dict(marks), end, [b.done for b in eng._shard.buckets] if eng._shard is not None else []))
        if eng._shard is not None:   # the bucket events are re-created every step: keep this step's
            for b in eng._shard.buckets:
                b.done = None
    torch.cuda.synchronize()
    out = []
    for mk, end, dones in rounds:
        t0 = mk["start"]
        rec = {"graph_end_ms": round(t0.elapsed_time(mk["graph_end"]), 3),
               "step_end_ms": round(t0.elapsed_time(end), 3)}
        if eng._shard is not None:
            rec["bucket_done_ms"] = [round(t0.elapsed_time(d), 3) for d in dones if d is not None]
            rec["bucket_params"] = [b.hi - b.lo for b in eng._shard.buckets]
            # > 0: the previous step's update of that bucket ended AFTER this step's forward started
            rec["prev_update_end_vs_forward_start_ms"] = {lo: round(t0.elapsed_time(ev), 3)
                                                          for lo, ev in mk["prev_ready"]}
            rec["staged_graphs"] = len(eng._ggraph) if isinstance(eng._ggraph, list) else 0
        out.append(rec)
    print(json.dumps({"overlap_env": os.environ.get("GARFIELD_OVERLAP", ""), "steps": out}), flush=True)


if __name__ == "__main__":
    main()
