"""GPU probe: how long does the slowdown of a graph on the main stream last after ONE
other stream waited on an event of the main stream? Times 40 consecutive replays after
a single cross-stream wait, then after a device-counter hand-off (parallel/signals.py)."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    dev = torch.device("cuda", 0)
    cap, side = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.randn(1 << 20, device=dev)
    b = torch.empty_like(a)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for i in range(400):
            (b if i % 2 else a).copy_(a if i % 2 else b)
    cur = torch.cuda.current_stream()
    tiny = torch.zeros(16, device=dev)
    out = {}
    for tag in ("event_wait", "none"):
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        if tag == "event_wait":
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                tiny.add_(1)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
        ev[0].record(cur)
        for i in range(40):
            g.replay()
            ev[i + 1].record(cur)
        torch.cuda.synchronize()
        out[tag] = [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(40)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
