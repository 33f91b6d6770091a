"""Tracing and profiling helpers.

Reference: ``--bench`` wraps a step in ``torch.autograd.profiler.profile`` and prints
``key_averages()`` (``Aggregathor/trainer.py:234-243``); Garfield_CC keeps hand
timers per phase (zero / gather / aggregate / flatten / reshape / broadcast,
``Garfield_CC/trainer.py:62-207``); ``tools.TimedContext`` times blocks.

Here:

* ``PhaseTimer`` — HIP-event timers per named phase (no host sync inside the step;
  ``summary()`` synchronises once), used by the engine's ``profile_phases`` option;
* ``range_push`` / ``range`` — roctx ranges (``torch.cuda.nvtx`` maps to roctx on
  ROCm), visible in ``rocprofv3 --marker-trace`` timelines;
* ``torch_profile`` — the reference's ``--bench`` behaviour (PyTorch profiler table).
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch


class PhaseTimer:
    """Accumulates device time per phase with HIP events (CPU wall time on CPU)."""

    def __init__(self, device, enabled: bool = True):
        self.device = torch.device(device)
        self.enabled = enabled
        self.cuda = self.device.type == "cuda"
        self._pending = []          # (name, start, end)
        self.totals = defaultdict(float)
        self.counts = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            with range_ctx(name):
                yield
            e.record()
            self._pending.append((name, s, e))
        else:
            import time

            t0 = time.perf_counter()
            yield
            self.totals[name] += 1000 * (time.perf_counter() - t0)
            self.counts[name] += 1

    def flush(self) -> None:
        if self._pending:
            torch.cuda.synchronize(self.device)
            for name, s, e in self._pending:
                self.totals[name] += s.elapsed_time(e)
                self.counts[name] += 1
            self._pending.clear()

    def summary(self) -> dict:
        """Mean milliseconds per call of every phase."""
        self.flush()
        return {k: self.totals[k] / max(self.counts[k], 1) for k in self.totals}

    def reset(self) -> None:
        self.flush()
        self.totals.clear()
        self.counts.clear()


def range_push(name: str) -> None:
    try:
        torch.cuda.nvtx.range_push(name)
    except Exception:
        pass


def range_pop() -> None:
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:
        pass


@contextlib.contextmanager
def range_ctx(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


@contextlib.contextmanager
def torch_profile(enabled: bool = True, sort_by: str = "self_cpu_time_total", row_limit: int = 25):
    """The reference's ``--bench`` profiler: prints the key-averages table on exit."""
    if not enabled:
        yield None
        return
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts) as prof:
        yield prof
    print(prof.key_averages().table(sort_by=sort_by, row_limit=row_limit))


def trace_graph(fn, what: str):
    """Wrap ``fn`` so each call prints ``[TRACE] (begin) what`` / ``[TRACE] (end)   what``
    around it and shows up as a named roctx range in ``rocprofv3 --marker-trace`` (reference
    ``TF/rsrcs/tools/tf.py:41-58``, which wires two ``tf.Print`` ops around a graph node).
    The end line is printed after the call returns on the host; GPU work it queued may
    still be running (use ``PhaseTimer`` for device time)."""
    import functools

    @functools.wraps(fn)
    def traced(*args, **kwargs):
        print(f"[TRACE] (begin) {what}", flush=True)
        with range_ctx(what):
            out = fn(*args, **kwargs)
        print(f"[TRACE] (end)   {what}", flush=True)
        return out

    return traced
