"""Host-side timing of the bench step: is the host ever blocked by the GPU inside a step?

Wraps the grouped graph replay, the aggregation/update and the whole ``eng.step`` call with
host timers (no device syncs added) and prints per-step host milliseconds. If a call's
host time is close to the step's device time, something in it waits for the GPU, and the
GPU idles while the host then issues the next step (the gap at each step boundary of
profiles/r2/rocprof_step_sequence_r2c.txt)."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import init_distributed  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402


def main():
    ctx = init_distributed()
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("resnet50", num_classes=10), F.cross_entropy, ctx,
                             EngineConfig(gar="krum", f=2, workers_per_rank=8, lr=0.01, momentum=0.9,
                                          weight_decay=5e-4, exchange_dtype=torch.bfloat16, cuda_graph=True,
                                          lp_weights=True, shard_gar=True if "--shard-gar" in sys.argv else None))
    batches = synthetic_batches(8, 250, (3, 32, 32), 10, ctx.device, seed=1)
    acc = {}

    def wrap(obj, name):
        fn = getattr(obj, name)

        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
            return r
        setattr(obj, name, w)

    for _ in range(4):
        eng.step(batches)
    torch.cuda.synchronize()
    wrap(eng, "_grouped_compute")
    wrap(eng, "aggregate_and_update")
    wrap(eng, "_stage_grouped")
    g = eng._ggraph
    for gg in (g if isinstance(g, list) else [g] if g is not None else []):
        wrap(gg, "replay")
    if eng._shard is not None:   # the sharded exchange's host calls (python bench: --shard-gar)
        for name in ("start_exchange", "_gather_bucket", "_gather_ranks", "_wait", "_finish_gathers"):
            wrap(eng._shard, name)
    steps = 20
    per = []
    t0 = time.perf_counter()
    for _ in range(steps):
        t = time.perf_counter()
        eng.step(batches)
        per.append(time.perf_counter() - t)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e3 * (t1 - t0) / steps:.3f} ms/step, drain {1e3 * (t2 - t1):.2f} ms, "
          f"wall {1e3 * (t2 - t0) / steps:.3f} ms/step")
    print("per-step host ms:", " ".join(f"{1e3 * p:.2f}" for p in per))
    print("host ms/step by call:", {k: round(1e3 * v / steps, 3) for k, v in acc.items()})


if __name__ == "__main__":
    main()
