"""Benchmark apps run end to end on CPU: collective bandwidth (gloo, 2 ranks), RPC
all-to-all pulls (3 local nodes) and the GAR micro-benchmark on host tensors."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    return dict(os.environ, PYTHONPATH=str(REPO), CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
                GARFIELD_NUM_THREADS="2")


def _rows(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def test_comm_bench_two_ranks():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(_port()), "-m", "garfield_amd.apps.comm_bench",
                        "--sizes", "4096", "65536", "--iters", "2", "--warmup", "1", "--dtype", "fp32"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    rows = _rows(r.stdout)
    assert {x["op"] for x in rows} == {"all_gather", "broadcast", "all_reduce", "all_to_all"}
    ag = [x for x in rows if x["op"] == "all_gather"][0]
    assert ag["world"] == 2 and ag["bytes"] == 2 * 4096 * 4 and ag["busbw_GBps"] > 0


def test_rpc_bench_spawn():
    r = subprocess.run([sys.executable, "-m", "garfield_amd.apps.rpc_bench", "--spawn", "--n", "3", "--d", "5000",
                        "--num_iter", "2", "--port", str(_port())], capture_output=True, text=True, timeout=300,
                       env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    rows = _rows(r.stdout)
    assert len(rows) == 6 and all(x["d"] == 5000 and x["n"] == 3 for x in rows)


def test_gar_bench_cpu():
    r = subprocess.run([sys.executable, "-m", "garfield_amd.apps.gar_bench", "--device", "cpu", "--n", "8",
                        "--d", "10000", "--iters", "1", "--rules", "krum", "median"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    rows = _rows(r.stdout)
    assert {x["rule"] for x in rows} == {"krum", "median"}


def test_bench_py_contract_two_ranks():
    """The driver's bench.py contract at world 2 (gloo): exactly one JSON line from rank 0
    with the required keys, n_gpus = WORLD_SIZE, weak scaling (k workers per rank)."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(REPO / "bench.py"),
                        "--gpus", "2", "--steps", "1", "--warmup", "1", "--model", "cifarnet", "--batch", "4",
                        "--workers-per-gpu", "3", "--f", "1"],
                       capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    rows = _rows(r.stdout)
    assert len(rows) == 1, r.stdout[-2000:]
    row = rows[0]
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in row, key
    assert row["n_gpus"] == 2 and row["steps"] == 1 and row["warmup"] == 1 and row["scaling"] == "weak"
    assert row["config"]["global_batch"] == 2 * 3 * 4 and row["value"] > 0
    assert row["replicas_identical"] and len(row["replica_checksums"]) == 2


def test_bench_py_self_launches_ranks():
    """``python bench.py --gpus 2`` with NO torchrun: bench.py starts torch.distributed.run
    itself (child process) and the JSON reports the real process-group size."""
    env = _env()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--model", "cifarnet", "--batch", "4", "--workers-per-gpu", "3", "--f", "1"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = _rows(r.stdout)
    assert len(rows) == 1, r.stdout[-2000:]
    assert rows[0]["n_gpus"] == 2 and rows[0]["config"]["global_batch"] == 2 * 3 * 4


def test_bench_py_rejects_world_mismatch():
    """A rank whose process group disagrees with --gpus must fail instead of printing a number."""
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--model", "cifarnet", "--batch", "2", "--workers-per-gpu", "3", "--f", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and not _rows(r.stdout)


def test_bench_py_fp32_and_static_data_modes():
    """--precision fp32 reports dtype fp32 (reference precision end to end); --data static and
    the default fresh-data feed both produce one JSON line with the data mode stated."""
    for extra, dtype, word in ((["--precision", "fp32"], "fp32", "fresh samples"),
                               (["--data", "static"], "bf16", "same batches")):
        r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--steps", "1", "--warmup", "1",
                            "--model", "cifarnet", "--batch", "4", "--workers-per-gpu", "5", "--f", "1", *extra],
                           capture_output=True, text=True, timeout=600, env=_env())
        assert r.returncode == 0, r.stderr[-3000:]
        rows = _rows(r.stdout)
        assert len(rows) == 1 and rows[0]["dtype"] == dtype and word in rows[0]["data"], rows


def test_bench_py_loss_is_a_training_signal():
    """The default fresh-data feed has learnable labels (class colour + noise, data/fresh.py):
    the loss of the last timed step is below the first warm-up step's and below ln(10)."""
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--steps", "30", "--warmup", "1",
                        "--model", "cifarnet", "--batch", "32", "--workers-per-gpu", "3", "--f", "0", "--gar",
                        "average", "--lr", "0.02"], capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    row = _rows(r.stdout)[0]
    assert row["final_loss"] < row["first_loss"] and row["final_loss"] < 2.3026, row
