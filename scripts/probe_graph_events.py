"""GPU probe: event-record / event-wait nodes attached to marker kernels of a captured
HIP graph (bindings.cpp graph_attach_*). Checks that another stream's wait on a
mark fires at the mark (not at the end of the graph), that a graph node can wait
for another stream's event, and what each costs.

    python scripts/probe_graph_events.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

C = _native.native()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
SPIN = 2_000_000   # cycles of torch.cuda._sleep (~1 ms at ~2 GHz)


def main():
    words = [C.signal_alloc(1) for _ in range(3)]
    evs = [C.event_create() for _ in range(3)]
    s = torch.cuda.Stream()
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=s):
        torch.cuda._sleep(SPIN)
        C.signal_set(words[0], 1, s.cuda_stream)
        torch.cuda._sleep(SPIN)
        C.signal_set(words[1], 1, s.cuda_stream)
        torch.cuda._sleep(SPIN)
    found = C.graph_attach_record_events(g.raw_cuda_graph(), words[:2], evs[:2], False)
    g.instantiate()
    res = {"markers_found": found}
    cur = torch.cuda.current_stream()
    for trial in range(5):
        t0 = torch.cuda.Event(enable_timing=True)
        t_end = torch.cuda.Event(enable_timing=True)
        t_m = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t0.record(cur)
        g.replay()
        t_end.record(cur)
        for i in range(2):
            C.event_wait(side.cuda_stream, evs[i])
            t_m[i].record(side)
        torch.cuda.synchronize()
        res.setdefault("record", []).append({"mark0_ms": round(t0.elapsed_time(t_m[0]), 3),
                                             "mark1_ms": round(t0.elapsed_time(t_m[1]), 3),
                                             "graph_end_ms": round(t0.elapsed_time(t_end), 3)})
    # wait node: the graph's second half waits for an event of another stream
    g2 = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g2, stream=s):
        torch.cuda._sleep(SPIN // 4)
        C.signal_set(words[2], 1, s.cuda_stream)
        torch.cuda._sleep(SPIN // 4)
    found2 = C.graph_attach_wait_events(g2.raw_cuda_graph(), [words[2]], [evs[2]], True)
    g2.instantiate()
    res["wait_markers_found"] = found2
    for trial in range(3):
        t0 = torch.cuda.Event(enable_timing=True)
        t_end = torch.cuda.Event(enable_timing=True)
        t_side = torch.cuda.Event(enable_timing=True)
        side.wait_stream(cur)
        t0.record(cur)
        with torch.cuda.stream(side):
            torch.cuda._sleep(4 * SPIN)
        C.event_record(evs[2], side.cuda_stream)
        t_side.record(side)
        g2.replay()
        t_end.record(cur)
        torch.cuda.synchronize()
        res.setdefault("wait", []).append({"side_done_ms": round(t0.elapsed_time(t_side), 3),
                                           "graph_end_ms": round(t0.elapsed_time(t_end), 3)})
    # cost: 200 tiny kernels with 8 marks, per variant (device time per replay, back to back)
    def build(variant):
        w8 = [C.signal_alloc(1) for _ in range(8)]
        e8 = [C.event_create() for _ in range(8)]
        if variant == "split":   # 8 graphs, eager event records between them
            gs = []
            for part in range(8):
                gp = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gp, stream=s):
                    for _ in range(25):
                        torch.cuda._sleep(100)
                gs.append(gp)

            def run():
                for i, gp in enumerate(gs):
                    gp.replay()
                    C.event_record(e8[i], torch.cuda.current_stream().cuda_stream)
                    C.event_wait(side.cuda_stream, e8[i])
            return run
        gg = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(gg, stream=s):
            for i in range(200):
                torch.cuda._sleep(100)
                if variant != "plain" and i % 25 == 24:
                    C.signal_set(w8[i // 25], 1, s.cuda_stream)
        if variant in ("inline", "leaf"):
            C.graph_attach_record_events(gg.raw_cuda_graph(), w8, e8, variant == "inline")
        gg.instantiate()

        def run():
            gg.replay()
            if variant in ("inline", "leaf"):
                for e in e8:
                    C.event_wait(side.cuda_stream, e)
        return run

    for variant in ("plain", "markers", "inline", "leaf", "split"):
        run = build(variant)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        a.record()
        for _ in range(50):
            run()
        b.record()
        torch.cuda.synchronize()
        res[variant + "_wall_ms"] = round((time.perf_counter() - t) * 1000 / 50, 4)
        res[variant + "_dev_ms"] = round(a.elapsed_time(b) / 50, 4)
    # inline record: does mark 0 fire at its point?
    gi = torch.cuda.CUDAGraph(keep_graph=True)
    wi = [C.signal_alloc(1) for _ in range(2)]
    ei = [C.event_create() for _ in range(2)]
    with torch.cuda.graph(gi, stream=s):
        torch.cuda._sleep(SPIN)
        C.signal_set(wi[0], 1, s.cuda_stream)
        torch.cuda._sleep(SPIN)
        C.signal_set(wi[1], 1, s.cuda_stream)
        torch.cuda._sleep(SPIN)
    C.graph_attach_record_events(gi.raw_cuda_graph(), wi, ei, True)
    gi.instantiate()
    for trial in range(3):
        t0 = torch.cuda.Event(enable_timing=True)
        t_end = torch.cuda.Event(enable_timing=True)
        t_m = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t0.record(cur)
        gi.replay()
        t_end.record(cur)
        for i in range(2):
            C.event_wait(side.cuda_stream, ei[i])
            t_m[i].record(side)
        torch.cuda.synchronize()
        res.setdefault("record_inline", []).append({"mark0_ms": round(t0.elapsed_time(t_m[0]), 3),
                                                    "mark1_ms": round(t0.elapsed_time(t_m[1]), 3),
                                                    "graph_end_ms": round(t0.elapsed_time(t_end), 3)})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
