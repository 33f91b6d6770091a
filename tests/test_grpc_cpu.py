"""gRPC transport (reference ``tensorflow_impl``): wire format, service semantics and
local multi-process AggregaThor / ByzSGD / LEARN clusters on 127.0.0.1 (CPU)."""
import json
import os
import socket
import subprocess
import sys
import threading
import time
from pathlib import Path

import numpy as np
import pytest

from garfield_amd.grpcnet import proto
from garfield_amd.grpcnet import service as S
from garfield_amd.grpcnet.aggregator import Aggregator
from garfield_amd.grpcnet.attacker import Attacker
from garfield_amd.grpcnet.network import Network, make_config, write_configs

REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_wire_format_matches_protoc_layout():
    # field numbers / types of the reference garfield.proto
    m = proto.Model(model=b"\x00\x01", init=True, iter=3)
    assert m.SerializeToString() == b"\n\x02\x00\x01\x10\x01\x18\x03"
    g = proto.Gradients(gradients=b"ab", iter=2.0)
    assert g.SerializeToString() == b"\n\x02ab\x15\x00\x00\x00@"
    r = proto.Request(iter=1, job="ps", req_id=4)
    assert proto.Request.FromString(r.SerializeToString()) == r


def test_history_bounded_and_blocking():
    h = S.History(keep=3)
    threading.Timer(0.2, lambda: h.append(np.ones(2, np.float32))).start()
    t0 = time.time()
    assert S.from_bytes(h.get(0, timeout=5)).tolist() == [1, 1]
    assert time.time() - t0 >= 0.15
    for _ in range(5):
        h.append(np.zeros(1, np.float32))
    with pytest.raises(S.Evicted):
        h.get(0, timeout=1)
    with pytest.raises(TimeoutError):
        h.get(100, timeout=0.1)
    assert len(h._data) == 3


def test_service_pull_quorum_and_push():
    services, servers, stubs = [], [], []
    for i in range(3):
        svc = S.MessageExchangeService(np.full(4, i, np.float32), wait_timeout=10)
        srv, port = S.make_server(svc, 0, host="127.0.0.1")
        srv.start()
        services.append(svc), servers.append(srv), stubs.append(S.Stub(f"127.0.0.1:{port}"))
    try:
        got = S.pull(stubs, "GetModel", 0, "worker", 0)
        assert sorted(int(a[0]) for _, a in got) == [0, 1, 2]
        # only peers 0 and 2 have gradient 0: a quorum of 2 returns without peer 1
        services[0].gradients_history.append(np.ones(2, np.float32))
        threading.Timer(0.2, lambda: services[2].gradients_history.append(np.full(2, 2, np.float32))).start()
        got = S.pull(stubs, "GetGradient", 0, "ps", 0, quorum=2)
        assert sorted(i for i, _ in got) == [0, 2]
        time.sleep(0.5)   # the straggling request to peer 1 was cancelled
        stubs[1].SendGradient(proto.Gradients(gradients=np.full(2, 9, np.float32).tobytes(), iter=0))
        assert S.pull([stubs[1]], "GetGradient", 0, "ps", 0)[0][1].tolist() == [9, 9]
        assert services[1].served("GetGradient", 0) == 1
    finally:
        for s in servers:
            s.stop(0)


def test_network_parser_and_generator(tmp_path):
    paths = write_configs(tmp_path, ["h:1", "h:2"], ["h:3"], "Median", "Krum", attacks={0: "Reverse"})
    assert len(paths) == 3
    n = Network(tmp_path / "TF_CONFIG_worker_0.json")
    assert n.get_task_type() == "worker" and n.get_my_attack() == "Reverse" and n.get_my_port() == "3"
    assert n.get_model_strategy() == "Median" and n.get_gradient_strategy() == "Krum"
    legacy = make_config(["h:1"], ["h:3"], "ps", 0)
    del legacy["task"]["strategy_model"], legacy["task"]["strategy_gradient"]
    legacy["task"]["strategy"] = "Bulyan"   # config_generator's key (bug B10)
    assert Network(data=legacy).get_gradient_strategy() == "Bulyan"


def test_attacker_and_aggregator_names():
    import torch

    g = torch.ones(1000)
    assert torch.equal(Attacker("Reverse").attack(g), -100 * g)
    dropped = Attacker("PartialDrop", probability=0.5).attack(g)
    assert 300 < int((dropped == 0).sum()) < 700
    lie = Attacker("LittleIsEnough").attack(g, [torch.zeros(1000)])
    assert torch.allclose(lie, torch.full((1000,), 0.5 + 1.035 * (0.5 ** 0.5)), atol=1e-5)
    rows = [np.random.RandomState(i).randn(50).astype(np.float32) for i in range(7)]
    rows[6] = rows[6] * 1e6
    out = Aggregator("Krum", 7, 1).aggregate(rows)
    assert isinstance(out, np.ndarray) and np.abs(out).max() < 100
    np.testing.assert_allclose(Aggregator("Average").aggregate(rows[:2]), (rows[0] + rows[1]) / 2, rtol=1e-6)
    with pytest.raises(AssertionError):
        Aggregator("Nope")


def _launch(cmds, tmp_path, timeout=240):
    env = dict(os.environ, PYTHONPATH=str(REPO), GARFIELD_NUM_THREADS="2", OMP_NUM_THREADS="1",
               CUDA_VISIBLE_DEVICES="")
    procs = []
    for i, c in enumerate(cmds):
        log = open(tmp_path / f"node{i}.log", "w")
        procs.append((subprocess.Popen([sys.executable, "-m", "garfield_amd.apps.grpc_trainer", *c], env=env,
                                       stdout=log, stderr=subprocess.STDOUT, cwd=tmp_path), log))
    deadline = time.time() + timeout
    try:
        for p, _ in procs:
            p.wait(timeout=max(deadline - time.time(), 1))
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
            log.close()
    for i, (p, _) in enumerate(procs):
        assert p.returncode == 0, (tmp_path / f"node{i}.log").read_text()[-3000:]


COMMON = ["--max_iter", "40", "--batch_size", "64", "--acc_freq", "39", "--linger", "30", "--retry_delay", "0.5"]


@pytest.mark.parametrize("app,num_ps,model_rule,grad_rule", [("aggregathor", 1, "Average", "Krum"),
                                                           ("byzsgd", 3, "Median", "Median")])
def test_grpc_cluster(tmp_path, app, num_ps, model_rule, grad_rule):
    workers = [f"127.0.0.1:{_free_port()}" for _ in range(5)]
    ps = [f"127.0.0.1:{_free_port()}" for _ in range(num_ps)]
    write_configs(tmp_path / "cfg", ps, workers, model_rule, grad_rule, attacks={4: "Reverse"})
    cmds = []
    for role, hosts in (("ps", ps), ("worker", workers)):
        for i in range(len(hosts)):
            cmds.append(["--app", app, "--config", str(tmp_path / "cfg" / f"TF_CONFIG_{role}_{i}.json"),
                         "--nbbyzwrks", "1", "--summary", str(tmp_path / f"{role}{i}.json"), *COMMON])
    _launch(cmds, tmp_path)
    accs = [json.loads((tmp_path / f"ps{i}.json").read_text())["accuracy"] for i in range(num_ps)]
    for a in accs:
        assert a[-1][1] > a[0][1] + 5, accs     # learns despite the reversed gradient
    if app == "byzsgd":   # replicas agree through the model median
        assert max(a[-1][1] for a in accs) - min(a[-1][1] for a in accs) < 5


def test_grpc_learn(tmp_path):
    n = 4
    ps = [f"127.0.0.1:{_free_port()}" for _ in range(n)]
    workers = [f"127.0.0.1:{_free_port()}" for _ in range(n)]
    write_configs(tmp_path / "cfg", ps, workers, "Median", "Median")
    cmds = [["--app", "learn", "--config_ps", str(tmp_path / "cfg" / f"TF_CONFIG_ps_{i}.json"),
             "--config_w", str(tmp_path / "cfg" / f"TF_CONFIG_worker_{i}.json"),
             "--summary", str(tmp_path / f"node{i}.json"), *COMMON] for i in range(n)]
    _launch(cmds, tmp_path)
    for i in range(n):
        acc = json.loads((tmp_path / f"node{i}.json").read_text())["accuracy"]
        assert acc[-1][1] > acc[0][1] + 5, acc


def test_legacy_train_message_exchange_service():
    """Every node also serves the reference's legacy TrainMessageExchange (all.proto):
    GetUnifiedModel / GetGradients / GetModel answer from the node's histories, the
    hash / signature methods are UNIMPLEMENTED (as in the reference), and the wire
    format follows all.proto's field numbers."""
    import grpc

    L = proto.LEGACY
    assert L["Gradients"](gradients=b"ab", iter=2.0, lipschitz=1.5).SerializeToString() == \
        b"\n\x02ab\x15\x00\x00\x00@\x1d\x00\x00\xc0?"
    assert L["Request"](iter=3, req_id=-1).SerializeToString() == b"\x08\x03\x10\xff\xff\xff\xff\xff\xff\xff\xff\xff\x01"
    base = S.MessageExchangeService(np.arange(4, dtype=np.float32), wait_timeout=10)
    server, port = S.make_server(base, 0, host="127.0.0.1")
    server.start()
    try:
        stub = S.LegacyStub(f"127.0.0.1:{port}")
        m = stub.GetUnifiedModel(L["Empty"](), timeout=10)
        assert m.init and S.from_bytes(m.model).tolist() == [0, 1, 2, 3]
        base.gradients_history.put(0, np.full(3, 7, np.float32))
        base.legacy.lipschitz[0] = 0.25
        g = stub.GetGradients(L["Request"](iter=0, req_id=5), timeout=10)
        assert S.from_bytes(g.gradients).tolist() == [7, 7, 7] and g.iter == 0 and g.lipschitz == 0.25
        assert base.served("GetGradient", 0) == 1
        base.model_weights_history.put(1, np.ones(2, np.float32))
        got = S.pull([stub], "GetModel", 1, "ps", -1)
        assert got[0][1].tolist() == [1, 1]
        with pytest.raises(grpc.RpcError) as e:
            stub.GetPublicKey(L["Empty"](), timeout=10)
        assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
        stub.close()
    finally:
        server.stop(0)
