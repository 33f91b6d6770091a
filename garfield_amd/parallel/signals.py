"""Stream-to-stream hand-offs that the HIP runtime does not see.

The exchange of a step runs on a side ("comm") stream: RCCL collectives, the bucket
packing, the simulated attacks. It must start when the main stream has produced its
input -- mid-way through the captured forward/backward graph (a bucket of layers is
complete), or after the main stream's GAR kernels. The obvious tool, an event recorded
on the main stream and waited for by the other stream, is what ROCm 7 makes
expensive on MI355X: once any other stream waits on an event of the main stream,
every later kernel of a graph replayed on the main stream runs ~1-1.5 us longer, and
the slowdown persists over several replays (``scripts/probe_cross_stream.py``,
``profiles/r3/probe_cross_stream.log``: a 400-kernel graph 0.88 -> 1.29-1.47 ms per
replay; a command-processor value wait, ``hipStreamWaitValue64``, 1.68 ms). torch's
ProcessGroupNCCL creates exactly that dependency (its internal stream waits on the
current stream) for every collective issued from the main stream.

``DeviceSignal`` is a 64-bit counter in device memory instead: ``record(stream)``
launches a 1-lane kernel that adds 1 with a system-scope release (captured into a graph
it fires once per replay); ``wait_on(stream)`` launches a 1-lane kernel that polls until
the counter reaches the number of records the host has issued so far (relaxed loads
with ``s_sleep``, then an acquire), bounded by a timeout that is counted as a miss
instead of hanging the queue. Same 400-kernel graph: 0.92 ms per replay. The reverse
direction (the main stream waiting on the comm stream) stays an ordinary event: it
costs nothing measurable (0.89 ms).
"""
from __future__ import annotations

import torch

from garfield_amd import _native

WAIT_TIMEOUT_US = 5_000_000   # a lost signal turns into a counted miss after 5 s, never a hang


class DeviceSignal:
    """A counter hand-off from the stream that ``record``s to the streams that ``wait_on`` it."""

    def __init__(self, device: torch.device):
        self._C = _native.native()
        self._t = torch.zeros(2, dtype=torch.int64, device=device)   # [counter, misses]
        self.target = 0          # records issued (eagerly, or by graph replays) so far

    def available(self) -> bool:
        return True

    def record(self, stream) -> None:
        """+1 on ``stream``. Inside a stream capture the kernel becomes a graph node that
        fires on every replay: the owner of the graph calls ``replayed()`` per replay."""
        self._C.signal_add(self._t.data_ptr(), stream.cuda_stream)
        if not torch.cuda.is_current_stream_capturing():
            self.target += 1

    def replayed(self, times: int = 1) -> None:
        self.target += times

    def wait_on(self, stream) -> None:
        """``stream`` waits (on the device) until every record issued so far has executed."""
        self._C.wait_geq(self._t.data_ptr(), self.target, WAIT_TIMEOUT_US, self._t.data_ptr() + 8,
                         stream.cuda_stream)

    def misses(self) -> int:
        """Waits that timed out (synchronises with the device)."""
        return int(self._t[1].item())


class Handoff:
    """main -> comm ordering for eager work: ``to_comm(main, comm)`` makes ``comm`` wait
    for everything issued on ``main`` so far (a DeviceSignal); the way back is an event."""

    def __init__(self, device: torch.device):
        self.sig = DeviceSignal(device)

    def to_comm(self, main, comm) -> None:
        self.sig.record(main)
        self.sig.wait_on(comm)

    @staticmethod
    def to_main(main, comm) -> None:
        main.wait_stream(comm)
