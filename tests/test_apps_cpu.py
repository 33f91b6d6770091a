"""Applications end-to-end on CPU, several processes on localhost (RPC / gloo).

BASELINE config 1 (MNIST MLP, 1 PS + 2 workers, CPU/gloo, average) is the first
test; datasets fall back to their synthetic twins offline."""
import os
import re
import socket
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(module, nranks, args, timeout=240):
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", GARFIELD_NUM_THREADS="2")
    # one log file per rank: sequentially draining pipes can block the other ranks
    logs = [tempfile.TemporaryFile(mode="w+") for _ in range(nranks)]
    procs = [subprocess.Popen([sys.executable, "-m", module, "--rank", str(r), "--port", str(port),
                               "--device", "cpu", *args], cwd=ROOT, env=env, stdout=logs[r],
                              stderr=subprocess.STDOUT, text=True) for r in range(nranks)]
    try:
        for p in procs:
            p.wait(timeout=timeout)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    outs = []
    for f in logs:
        f.seek(0)
        outs.append(f.read())
        f.close()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    return outs


def accuracies(text):
    return [float(x) for x in re.findall(r"Accuracy: ([0-9.]+)", text)]


def test_aggregathor_plumbing_config1():
    outs = run_ranks("garfield_amd.apps.aggregathor", 3,
                     ["--num_workers", "2", "--model", "mlp", "--dataset", "mnist", "--num_iter", "40",
                      "--acc_freq", "20", "--gar", "average", "--batch", "32"])
    acc = accuracies(outs[0])
    assert len(acc) >= 2 and acc[-1] > acc[0]


def test_aggregathor_krum_with_byzantine_worker():
    # the server waits for the fastest n - fw = 5 gradients: Krum(f=1) needs >= 2f + 3 = 5
    outs = run_ranks("garfield_amd.apps.aggregathor", 7,
                     ["--num_workers", "6", "--fw", "1", "--attack", "reverse", "--gar", "krum", "--model", "mlp",
                      "--dataset", "mnist", "--num_iter", "30", "--acc_freq", "15", "--batch", "16"])
    acc = accuracies(outs[0])
    assert acc[-1] > acc[0]


def test_byzsgd_byzantine_server_and_worker():
    # 4 servers (server 0 Byzantine) / 4 workers (worker 0 Byzantine); every server waits for the
    # fastest 3 gradients and 3 models: the median of 3 tolerates one Byzantine input
    outs = run_ranks("garfield_amd.apps.byzsgd", 8,
                     ["--num_ps", "4", "--num_workers", "4", "--fw", "1", "--fps", "1", "--gar", "median",
                      "--attack", "reverse", "--model", "mlp", "--dataset", "mnist", "--num_iter", "30",
                      "--acc_freq", "15", "--opt_args", '{"lr": "0.05"}'])
    acc = accuracies(outs[1])
    assert acc[-1] > acc[0]


def test_learn_non_iid():
    outs = run_ranks("garfield_amd.apps.learn", 3,
                     ["--num_nodes", "3", "--f", "0", "--gar", "average", "--model", "mlp", "--dataset", "mnist",
                      "--num_iter", "12", "--acc_freq", "6", "--non_iid", "1"])
    assert accuracies(outs[0])


def test_centralized():
    out = subprocess.run([sys.executable, "-m", "garfield_amd.apps.centralized", "--model", "mlp", "--dataset",
                          "mnist", "--num_iter", "30", "--acc_freq", "15", "--device", "cpu"], cwd=ROOT,
                         env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    acc = accuracies(out.stdout)
    assert acc[-1] > acc[0]


def test_garfield_cc_byzantine_servers():
    """BASELINE config 5 shape on CPU: 3 server replicas + 5 workers, fps = fw = 1, trimmed mean."""
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "8", "--master-addr",
                          "127.0.0.1", "--master-port", str(port), "-m", "garfield_amd.apps.garfield_cc",
                          "--num_ps", "3", "--fps", "1", "--fw", "1", "--attack", "reverse", "--ps_attack", "reverse",
                          "--aggregator", "trimmed-mean", "--mar", "trimmed-mean", "--model", "mlp", "--dataset",
                          "mnist", "--num_iter", "30", "--lr", "0.05", "--loss", "nll"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    m = re.search(r"final accuracy ([0-9.]+)", out.stdout + out.stderr)
    assert m and float(m.group(1)) > 15.0


def test_garfield_cc_crash_mar():
    """--mar crash (reference Garfield_CC/trainer.py:97,137,520-523): 2 trusted servers + 2 workers,
    median gradient aggregation, servers averaged (their aggregates are identical)."""
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    base = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
            "--master-port", str(port), "-m", "garfield_amd.apps.garfield_cc", "--num_ps", "2",
            "--aggregator", "median", "--model", "mlp", "--dataset", "mnist", "--num_iter", "10", "--lr", "0.05",
            "--loss", "nll", "--workers_per_rank", "3", "--mar", "crash"]
    out = subprocess.run(base, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    assert re.search(r"final accuracy ([0-9.]+)", out.stdout + out.stderr)


def test_garfield_cc_checkpoint_resume_is_exact(tmp_path):
    """2 ranks (gloo): 6 iterations straight == 3 iterations, checkpoint, fresh processes
    resuming from it for the last 3 (parameters, momentum, BatchNorm buffers, step)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")

    def run(extra):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
               "127.0.0.1", "--master-port", str(free_port()), "-m", "garfield_amd.apps.garfield_cc",
               "--model", "mlp", "--dataset", "mnist", "--loss", "nll", "--lr", "0.05", "--aggregator", "krum",
               "--fw", "1", "--attack", "reverse", "--workers_per_rank", "3", *extra]
        out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
        return re.search(r"replica checksum ([-+0-9.e]+)", out.stdout + out.stderr).group(1)

    straight = run(["--num_iter", "6"])
    ck = str(tmp_path / "ck")
    run(["--num_iter", "3", "--checkpoint", ck, "--checkpoint_freq", "3"])
    resumed = run(["--num_iter", "6", "--checkpoint", ck, "--resume", "1"])
    assert resumed == straight


def test_garfield_cc_layerwise():
    """--layerwise: the GAR per parameter tensor (reference Garfield_CC semantics), 2 ranks."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), "-m", "garfield_amd.apps.garfield_cc", "--model", "mlp", "--dataset",
           "mnist", "--loss", "nll", "--lr", "0.05", "--aggregator", "krum", "--fw", "1", "--attack", "reverse",
           "--workers_per_rank", "3", "--num_iter", "10", "--layerwise", "1"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    assert re.search(r"final accuracy ([0-9.]+)", out.stdout + out.stderr)


def test_garfield_cc_byzantine_servers_hosting_workers():
    """--ps_workers: the 3 server ranks also train (8 ranks x 2 logical workers, fw = 2 of 16)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "8", "--master-addr",
                          "127.0.0.1", "--master-port", str(free_port()), "-m", "garfield_amd.apps.garfield_cc",
                          "--num_ps", "3", "--fps", "1", "--fw", "2", "--attack", "reverse", "--ps_attack", "reverse",
                          "--ps_workers", "1", "--workers_per_rank", "2", "--aggregator", "trimmed-mean", "--mar",
                          "trimmed-mean", "--model", "mlp", "--dataset", "mnist", "--num_iter", "30", "--lr", "0.05",
                          "--loss", "nll"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    m = re.search(r"final accuracy ([0-9.]+)", out.stdout + out.stderr)
    assert m and float(m.group(1)) > 15.0


def test_garfield_cc_fastest_quorum_with_straggler():
    """--quorum 2 of 3 ranks with rank 2 delayed (fault injection): the run completes and
    prints one replica checksum (all replicas applied the leader's quorum sets)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "3", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), "-m", "garfield_amd.apps.garfield_cc", "--model", "mlp", "--dataset",
           "mnist", "--loss", "nll", "--lr", "0.05", "--aggregator", "median", "--fw", "1", "--attack", "reverse",
           "--workers_per_rank", "2", "--num_iter", "8", "--quorum", "2", "--straggler", "2:0.3"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    assert re.search(r"final accuracy ([0-9.]+)", out.stdout + out.stderr)


def test_garfield_cc_multistep_lr_schedule():
    """The reference's per-epoch MultiStepLR (Garfield_CC trainer.py:273-274,290-291: milestones [25, 50],
    gamma 0.1 for resnet50, stepped at each epoch's start) drives the engine's fused update."""
    from garfield_amd.apps import garfield_cc

    assert [garfield_cc.multistep_lr(0.2, [25, 50], 0.1, e) for e in (0, 23, 24, 48, 49, 80)] == \
        pytest.approx([0.2, 0.2, 0.02, 0.02, 0.002, 0.002])
    res = {}
    garfield_cc.main(["--model", "pimanet", "--dataset", "pima", "--loss", "binary-cross-entropy", "--batch", "200",
                      "--epochs", "3", "--lr", "0.1", "--lr_milestones", "2,3", "--cuda_graph", "0"], results=res)
    assert res["lrs"] == pytest.approx([0.1, 0.01, 0.001])
