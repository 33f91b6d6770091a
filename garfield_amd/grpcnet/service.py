"""``MessageExchange`` gRPC service, server and client (the TF transport).

Reference: ``tensorflow_impl/libs/grpc_message_exchange_servicer.py:33-90`` (servicer),
``libs/server.py:83-143`` (server + pull loops), ``libs/tools.py:146-159``
(``set_connection``). Differences, on purpose:

* the per-iteration history is a **bounded** ring (``keep`` iterations, default 64)
  instead of an ever-growing list (bug B13), and readers block on a condition
  variable instead of a 1 ms busy-wait;
* ``SendModel`` / ``SendGradient`` are implemented (push mode; the reference
  answers UNIMPLEMENTED), so a node can also be fed by its peers;
* a pull from many peers is issued concurrently (one future per peer) and can stop
  at the fastest ``q`` replies (the async quorum of ``pytorch_impl/libs/garfieldpp/
  server.py:134-155``), rather than one blocking call after another;
* a request for an iteration that is already evicted fails with OUT_OF_RANGE
  instead of hanging; a request that waits longer than ``wait_timeout`` fails with
  DEADLINE_EXCEEDED so that the client's retry loop takes over.

Payloads are flat little-endian fp32 vectors (``np.float32.tobytes()``), the
reference's interchange layout.
"""
from __future__ import annotations

import threading
import time
from concurrent import futures

import grpc
import numpy as np

from garfield_amd.grpcnet import proto

MAX_MESSAGE = -1   # unlimited (reference: 500 MB on the server, unlimited on the client)
GRPC_OPTIONS = [("grpc.max_send_message_length", MAX_MESSAGE), ("grpc.max_receive_message_length", MAX_MESSAGE)]


class Evicted(KeyError):
    pass


class History:
    """Iteration-indexed payload store: ``append`` commits iteration ``len(self)``;
    ``put`` stores an explicit iteration (push mode); ``get`` blocks until present."""

    def __init__(self, keep: int = 64):
        self.keep = max(int(keep), 1)
        self._data: dict[int, bytes] = {}
        self._next = 0
        self._cv = threading.Condition()

    def __len__(self) -> int:
        with self._cv:
            return self._next

    def _evict(self) -> None:
        low = self._next - self.keep
        for k in [k for k in self._data if k < low]:
            del self._data[k]

    def append(self, payload) -> int:
        data = to_bytes(payload)
        with self._cv:
            it = self._next
            self._data[it] = data
            self._next += 1
            self._evict()
            self._cv.notify_all()
            return it

    def put(self, it: int, payload) -> None:
        data = to_bytes(payload)
        with self._cv:
            self._data[int(it)] = data
            self._next = max(self._next, int(it) + 1)
            self._evict()
            self._cv.notify_all()

    def get(self, it: int, timeout: float | None = None) -> bytes:
        it = int(it)
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while it not in self._data:
                if it < self._next - self.keep:
                    raise Evicted(it)
                remaining = None if deadline is None else deadline - time.monotonic()
                if remaining is not None and remaining <= 0:
                    raise TimeoutError(it)
                self._cv.wait(remaining)
            return self._data[it]


def to_bytes(payload) -> bytes:
    if isinstance(payload, bytes):
        return payload
    if hasattr(payload, "detach"):       # torch tensor (any device)
        payload = payload.detach().reshape(-1).float().cpu().numpy()
    return np.ascontiguousarray(payload, dtype=np.float32).tobytes()


def from_bytes(data: bytes) -> np.ndarray:
    return np.frombuffer(data, dtype=np.float32)


class MessageExchangeService:
    """Server-side handlers; ``model_weights_history`` starts with the initial model."""

    def __init__(self, model_weights=None, keep: int = 64, wait_timeout: float = 120.0):
        self.model_weights_history = History(keep)
        self.gradients_history = History(keep)
        self.wait_timeout = wait_timeout
        self._served: dict[tuple[str, int], int] = {}
        self._served_cv = threading.Condition()
        if model_weights is not None:
            self.model_weights_history.append(model_weights)

    def _mark(self, method: str, it: int) -> None:
        with self._served_cv:
            self._served[(method, it)] = self._served.get((method, it), 0) + 1
            self._served_cv.notify_all()

    def served(self, method: str, it: int) -> int:
        with self._served_cv:
            return self._served.get((method, int(it)), 0)

    def wait_served(self, method: str, it: int, count: int, timeout: float) -> bool:
        """Block until ``method`` answered iteration ``it`` ``count`` times (used to
        keep a node serving until its peers pulled the last iteration)."""
        with self._served_cv:
            return self._served_cv.wait_for(lambda: self._served.get((method, int(it)), 0) >= count, timeout)

    def _get(self, hist: History, it: int, context):
        """Wait (in 0.5 s slices, so a cancelled client frees the handler thread)."""
        deadline = time.monotonic() + self.wait_timeout
        while True:
            try:
                return hist.get(it, min(0.5, max(deadline - time.monotonic(), 0.0)))
            except Evicted:
                context.abort(grpc.StatusCode.OUT_OF_RANGE, f"iteration {it} is no longer kept")
            except TimeoutError:
                if not context.is_active():
                    return None
                if time.monotonic() >= deadline:
                    context.abort(grpc.StatusCode.DEADLINE_EXCEEDED, f"iteration {it} not available yet")

    def GetModel(self, request, context):
        data = self._get(self.model_weights_history, request.iter, context)
        if data is None or not context.is_active():
            return proto.Model()
        self._mark("GetModel", request.iter)
        return proto.Model(model=data, init=True, iter=request.iter)

    def SendModel(self, request, context):
        self.model_weights_history.put(request.iter, request.model)
        return proto.Response(iter=request.iter, job="model")

    def GetGradient(self, request, context):
        data = self._get(self.gradients_history, request.iter, context)
        if data is None or not context.is_active():
            return proto.Gradients()
        self._mark("GetGradient", request.iter)
        return proto.Gradients(gradients=data, iter=float(request.iter))

    def SendGradient(self, request, context):
        it = int(request.iter)
        self.gradients_history.put(it, request.gradients)
        return proto.Response(iter=it, job="gradient")


class TrainMessageExchangeService:
    """The legacy ``TrainMessageExchange`` service (reference
    ``Garfield_legacy/all.proto:5-65``, ``grpc_service_impl.py:42-66``) over a node's
    MessageExchangeService histories:

    * ``GetUnifiedModel(Empty)``: the initial model (model history entry 0);
    * ``GetGradients(Request)``: gradient history entry ``iter`` -- a worker's gradient,
      or the aggregated gradient a PS published for that iteration -- with the
      Lipschitz value the node recorded for it (``lipschitz``, 0 if none);
    * ``GetModel(Request)``: model history entry ``iter`` (the PS-to-PS exchange).

    The hash / signature / public-key methods were never implemented by the reference
    either; they answer UNIMPLEMENTED."""

    def __init__(self, base: MessageExchangeService):
        self.base = base
        self.lipschitz: dict[int, float] = {}

    def GetUnifiedModel(self, request, context):
        b = self.base
        data = b._get(b.model_weights_history, 0, context)
        if data is None or not context.is_active():
            return proto.LEGACY["Model"]()
        b._mark("GetModel", 0)
        return proto.LEGACY["Model"](model=data, init=True, iter=0)

    def GetGradients(self, request, context):
        b = self.base
        data = b._get(b.gradients_history, request.iter, context)
        if data is None or not context.is_active():
            return proto.LEGACY["Gradients"]()
        b._mark("GetGradient", request.iter)
        return proto.LEGACY["Gradients"](gradients=data, iter=float(request.iter),
                                           lipschitz=float(self.lipschitz.get(int(request.iter), 0.0)))

    def GetModel(self, request, context):
        b = self.base
        data = b._get(b.model_weights_history, request.iter, context)
        if data is None or not context.is_active():
            return proto.LEGACY["Model"]()
        b._mark("GetModel", request.iter)
        return proto.LEGACY["Model"](model=data, init=True, iter=request.iter)

    def _unimplemented(self, request, context):
        context.abort(grpc.StatusCode.UNIMPLEMENTED, "not implemented (as in the reference)")

    GetPublicKey = GetCompleteModel = GetOnlyHash = GetGradHashes = GetGradHash = _unimplemented


def _handlers(impl, methods, classes) -> dict:
    return {meth: grpc.unary_unary_rpc_method_handler(getattr(impl, meth), request_deserializer=classes[req].FromString,
                                                      response_serializer=classes[resp].SerializeToString)
            for meth, req, resp in methods}


def make_server(service: MessageExchangeService, port: int | str, max_workers: int = 30,
                host: str | None = None) -> tuple[grpc.Server, int]:
    """gRPC server exposing ``service`` on ``host:port`` (port 0 → any free port), as
    ``MessageExchange`` and as the legacy ``TrainMessageExchange`` (``service.legacy``)."""
    service.legacy = TrainMessageExchangeService(service)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=GRPC_OPTIONS)
    server.add_generic_rpc_handlers((
        grpc.method_handlers_generic_handler(proto.SERVICE, _handlers(service, proto.METHODS, proto.CLASSES)),
        grpc.method_handlers_generic_handler(proto.LEGACY_SERVICE, _handlers(service.legacy, proto.LEGACY_METHODS,
                                                                             proto.LEGACY))))
    for h in ([host] if host else ["[::]", "0.0.0.0"]):
        try:
            bound = server.add_insecure_port(f"{h}:{port}")
        except RuntimeError:
            bound = 0
        if bound:
            return server, bound
    raise OSError(f"cannot bind the gRPC server to port {port}")


class Stub:
    """Client of one peer (reference ``tools.set_connection``)."""

    def __init__(self, target: str):
        self.target = target
        self.channel = grpc.insecure_channel(target, options=GRPC_OPTIONS)
        for meth, req, resp in proto.METHODS:
            setattr(self, meth, self.channel.unary_unary(
                f"/{proto.SERVICE}/{meth}", request_serializer=proto.CLASSES[req].SerializeToString,
                response_deserializer=proto.CLASSES[resp].FromString))

    def close(self) -> None:
        self.channel.close()

    @staticmethod
    def request(method: str, it: int, job: str, req_id: int):
        return proto.Request(iter=int(it), job=job, req_id=int(req_id))


class LegacyStub(Stub):
    """Client of a peer's ``TrainMessageExchange`` service (legacy Garfield clients)."""

    def __init__(self, target: str):
        self.target = target
        self.channel = grpc.insecure_channel(target, options=GRPC_OPTIONS)
        for meth, req, resp in proto.LEGACY_METHODS:
            setattr(self, meth, self.channel.unary_unary(
                f"/{proto.LEGACY_SERVICE}/{meth}", request_serializer=proto.LEGACY[req].SerializeToString,
                response_deserializer=proto.LEGACY[resp].FromString))

    @staticmethod
    def request(method: str, it: int, job: str, req_id: int):
        if method in ("GetUnifiedModel", "GetPublicKey"):
            return proto.LEGACY["Empty"]()
        return proto.LEGACY["Request"](iter=int(it), req_id=int(req_id))


def set_connection(host: str) -> Stub:
    return Stub(host)


def _payload(resp) -> bytes:
    return resp.model if resp.DESCRIPTOR.name == "Model" else resp.gradients


def pull(stubs: list[Stub], method: str, it: int, job: str, req_id: int, quorum: int | None = None,
         retries: int = 10, retry_delay: float = 5.0, timeout: float = 300.0) -> list[tuple[int, np.ndarray]]:
    """Concurrent ``method`` (GetModel / GetGradient; on ``LegacyStub``s GetUnifiedModel /
    GetGradients / GetModel) on every stub; returns the first
    ``quorum`` replies (all by default) as ``(peer_index, fp32 vector)`` in arrival
    order. Failed peers are retried ``retries`` times with ``retry_delay`` seconds
    between attempts (reference: 5 s sleeps, 10 or 100 attempts)."""
    n = len(stubs)
    q = n if quorum is None or quorum < 0 else min(int(quorum), n)
    done: list[tuple[int, np.ndarray]] = []
    failed: dict[int, Exception] = {}
    cv = threading.Condition()
    attempts = [0] * n
    pending: dict[int, object] = {}

    def launch(i):
        with cv:
            if len(done) >= q:
                return
            req = stubs[i].request(method, it, job, req_id)
            fut = getattr(stubs[i], method).future(req, timeout=timeout, wait_for_ready=True)
            pending[i] = fut
        fut.add_done_callback(lambda f, i=i: on_done(i, f))

    def on_done(i, fut):
        try:
            data = from_bytes(_payload(fut.result()))
        except Exception as e:  # noqa: BLE001 - grpc.RpcError or cancellation
            with cv:
                if len(done) >= q:
                    return
                attempts[i] += 1
                fatal = isinstance(e, grpc.RpcError) and e.code() == grpc.StatusCode.OUT_OF_RANGE
                if fatal or attempts[i] > retries:
                    failed[i] = e
                    cv.notify_all()
                    return
            threading.Timer(retry_delay, launch, (i,)).start()
            return
        with cv:
            if len(done) < q:
                done.append((i, data))
            cv.notify_all()

    for i in range(n):
        launch(i)
    with cv:
        while len(done) < q:
            if len(failed) > n - q:
                errs = "; ".join(f"{stubs[i].target}: {e}" for i, e in failed.items())
                raise ConnectionError(f"{method}({it}): fewer than {q} of {n} peers answered ({errs})")
            cv.wait(1.0)
        result = list(done[:q])
        stragglers = [f for i, f in pending.items() if i not in {j for j, _ in result}]
    for f in stragglers:   # the quorum is reached: stop waiting for the slowest peers
        f.cancel()
    return result
