"""Garfield_legacy protocol (TF1 byzPS/byzWorker) over gRPC on 127.0.0.1: vanilla,
asyncr and smart modes learn, with a Byzantine worker and the Kardam filter."""
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest
import torch

from garfield_amd.data.datasets import poison_batch
from garfield_amd.grpcnet.network import write_configs
from garfield_amd.runtime.kardam import LipschitzFilter

REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(cmds, tmp_path, timeout=300):
    env = dict(os.environ, PYTHONPATH=str(REPO), GARFIELD_NUM_THREADS="2", OMP_NUM_THREADS="1",
               CUDA_VISIBLE_DEVICES="")
    procs = []
    for i, c in enumerate(cmds):
        log = open(tmp_path / f"node{i}.log", "w")
        procs.append((subprocess.Popen([sys.executable, "-m", "garfield_amd.apps.legacy", *c], env=env,
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


@pytest.mark.parametrize("mode,num_ps,nbbyzps,attack", [("--vanilla", 1, 0, None), ("--asyncr", 3, 0, "Reverse"),
                                                       ("--smart", 3, 0, "Reverse")])
def test_legacy_cluster_learns(tmp_path, mode, num_ps, nbbyzps, attack):
    workers = [f"127.0.0.1:{_free_port()}" for _ in range(5)]
    ps = [f"127.0.0.1:{_free_port()}" for _ in range(num_ps)]
    write_configs(tmp_path / "cfg", ps, workers, "Median", "Krum", attacks={4: attack} if attack else {})
    common = [mode, "--max_steps", "40", "--batch", "64", "--eval_steps", "39", "--linger", "60", "--retry_delay",
              "0.5", "--nbbyzps", str(nbbyzps), "--T", "10"]
    if attack:
        common += ["--nbbyzwrk", "1"]
    cmds = []
    for role, hosts in (("ps", ps), ("worker", workers)):
        for i in range(len(hosts)):
            cmds.append(["--config", str(tmp_path / "cfg" / f"TF_CONFIG_{role}_{i}.json"),
                         "--summary", str(tmp_path / f"{role}{i}.json"), *common])
    _launch(cmds, tmp_path)
    for i in range(num_ps):
        acc = json.loads((tmp_path / f"ps{i}.json").read_text())["accuracy"]
        assert acc[-1][1] > acc[0][1] + 5, acc
    if mode == "--smart":
        k = json.loads((tmp_path / "worker0.json").read_text())["kardam"]
        assert k["observed"] == 39


def test_lipschitz_filter():
    f = LipschitzFilter(num_ps=3, num_byz_ps=1)
    assert f.observe(torch.ones(4), torch.zeros(4)) is None
    for t in range(1, 20):
        st = f.observe(torch.ones(4) * (1 + 0.01 * t), torch.full((4,), 0.1 * t))
    assert st is not None and abs(st.lipschitz - 0.1) < 1e-4
    st = f.observe(torch.ones(4) * (1.19 + 0.001), torch.full((4,), 2.0))   # smooth step: L = 0.01
    assert st.accept
    st = f.observe(torch.full((4,), 1e6), torch.full((4,), 2.1))     # a huge jump in gradient
    assert not st.accept and f.rejected >= 1


def test_poison_batch():
    x, y = torch.ones(8, 3), torch.arange(8)
    x1, y1 = poison_batch(x, y, 1)
    assert torch.equal(x1, -100 * x) and torch.equal(y1, y)
    x2, y2 = poison_batch(x, y, 2, torch.Generator().manual_seed(0))
    assert torch.equal(x2, -1e12 * x) and sorted(y2.tolist()) == list(range(8))
