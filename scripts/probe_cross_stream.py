"""GPU probe: what a cross-stream dependency costs a HIP graph replayed on the main stream.

Observed in the bucketed step (scripts/gpu_r3_streams.sh): when another stream waits on
an event recorded on the main stream right after the grouped step's graph, the graph
itself runs ~0.15 ms longer. This replays a graph of many small kernels in a loop and
times each variant with events on the main stream (device time per replay).

    python scripts/probe_cross_stream.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

C = _native.native()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
NK = int(os.environ.get("NK", "400"))


def main():
    cap = torch.cuda.Stream()
    side = torch.cuda.Stream()
    a = torch.randn(1 << 20, device=dev)
    b = torch.empty_like(a)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for i in range(NK):
            (b if i % 2 else a).copy_(a if i % 2 else b)   # ~3-5 us memory-bound kernels
    cur = torch.cuda.current_stream()
    tiny = torch.zeros(16, device=dev)
    ev = C.event_create()
    res = {}

    def variant(name, fn, iters=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record(cur)
        for _ in range(iters):
            fn()
        t1.record(cur)
        torch.cuda.synchronize()
        res[name] = round(t0.elapsed_time(t1) / iters, 4)

    def v_plain():
        g.replay()

    def v_side_waits_main():
        g.replay()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            tiny.add_(1)

    def v_side_waits_after_kernel():
        g.replay()
        tiny.add_(1)                      # an eager kernel between the graph and the recorded event
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            tiny.mul_(1)

    def v_main_waits_side():
        with torch.cuda.stream(side):
            tiny.add_(1)
        g.replay()
        cur.wait_stream(side)

    def v_native_event():
        g.replay()
        C.event_record(ev, cur.cuda_stream)
        C.event_wait(side.cuda_stream, ev)
        with torch.cuda.stream(side):
            tiny.add_(1)

    def v_side_waits_before_graph():
        side.wait_stream(cur)             # the wait targets the work BEFORE the graph
        with torch.cuda.stream(side):
            tiny.add_(1)
        g.replay()

    evs = {k: C.event_create(k) for k in (0, 1, 2)}

    def v_scoped(k):
        def f():
            g.replay()
            C.event_record(evs[k], cur.cuda_stream)
            C.event_wait(side.cuda_stream, evs[k])
            with torch.cuda.stream(side):
                tiny.add_(1)
        return f

    def v_record_no_waiter():
        g.replay()
        torch.cuda.Event().record(cur)

    state = {"i": 0}

    def v_wait_once_then_plain():   # one cross-stream wait every 5 replays: does the penalty persist?
        g.replay()
        state["i"] += 1
        if state["i"] % 5 == 0:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                tiny.add_(1)

    cnt_t = torch.zeros(2, dtype=torch.int64, device=dev)   # [counter, miss count] in device memory
    cnt, err = cnt_t.data_ptr(), cnt_t.data_ptr() + 8
    st = {"n": 0}

    def v_device_flag():           # main: +1 marker after the graph; side: bounded device-side wait
        g.replay()
        C.signal_add(cnt, cur.cuda_stream)
        st["n"] += 1
        C.wait_geq(cnt, st["n"], 2_000_000, err, side.cuda_stream)
        with torch.cuda.stream(side):
            tiny.add_(1)

    wv = C.signal_alloc(1)
    st2 = {"n": 0}

    def v_cp_value_wait():         # main: marker sets a value; side: command-processor wait
        st2["n"] += 1
        g.replay()
        C.signal_set(wv, st2["n"], cur.cuda_stream)
        C.stream_wait_value(side.cuda_stream, wv, st2["n"])
        with torch.cuda.stream(side):
            tiny.add_(1)

    def v_side_sleep():           # an unrelated 1-wave kernel running on the side stream meanwhile
        with torch.cuda.stream(side):
            torch.cuda._sleep(2_000_000)
        g.replay()
        cur.wait_stream(side)

    def v_side_sleep_after():     # the same kernel, but queued after the graph on the main stream
        g.replay()
        torch.cuda._sleep(2_000_000)

    side2 = torch.cuda.Stream()

    def v_device_flag_chain():     # + a third stream waiting (HIP event) on the side stream, as RCCL's would
        g.replay()
        C.signal_add(cnt, cur.cuda_stream)
        st["n"] += 1
        C.wait_geq(cnt, st["n"], 2_000_000, err, side.cuda_stream)
        with torch.cuda.stream(side):
            tiny.add_(1)
        side2.wait_stream(side)
        with torch.cuda.stream(side2):
            tiny.mul_(1)
        cur.wait_stream(side2)

    variant("device_flag_chain", v_device_flag_chain)
    variant("side_sleep_concurrent", v_side_sleep, iters=10)
    variant("sleep_serial", v_side_sleep_after, iters=10)
    variant("device_flag", v_device_flag)
    variant("cp_value_wait", v_cp_value_wait)
    torch.cuda.synchronize()
    res["device_flag_misses"] = int(cnt_t[1])
    for name, fn in (("scope0_system", v_scoped(0)), ("scope1_device", v_scoped(1)), ("scope2_nofence", v_scoped(2)),
                     ("record_no_waiter", v_record_no_waiter), ("wait_every_5th", v_wait_once_then_plain)):
        variant(name, fn)
    for name, fn in (("plain", v_plain), ("side_waits_main", v_side_waits_main),
                     ("side_waits_after_kernel", v_side_waits_after_kernel), ("main_waits_side", v_main_waits_side),
                     ("native_event", v_native_event), ("side_waits_before_graph", v_side_waits_before_graph),
                     ("plain_again", v_plain)):
        variant(name, fn)
    print(json.dumps({"kernels_per_graph": NK, "ms_per_replay": res}), flush=True)


if __name__ == "__main__":
    main()
