"""Reference import names (compat/): a script written against the reference's
``pytorch_impl/libs`` (``garfieldpp``, ``aggregators``, ``native``, ``tools`` on
sys.path) runs unchanged on Garfield-MI355X. Runs in a subprocess so the generic
top-level names (``tools``, ``native``) never shadow anything in the test process."""
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

SCRIPT = r'''
import torch
import aggregators, native, tools
from garfieldpp.worker import Worker
from garfieldpp.byzWorker import ByzWorker
from garfieldpp.server import Server
from garfieldpp import tools as gtools, datasets, models

torch.manual_seed(0)
g = [torch.randn(50) for _ in range(7)]
g[6] = g[6] * -100.0
out = aggregators.gars["native-krum"](gradients=g, f=2)
assert out.shape == (50,) and torch.isfinite(out).all()
assert aggregators.gars["krum"].check(gradients=g, f=2) is None
assert aggregators.gars["krum"].check(gradients=g[:4], f=2) is not None       # n < 2f + 3
b = native.bulyan.aggregate(g[:7], 1, 4)
assert b.shape == (50,)
m = native.median.aggregate(g)
assert torch.equal(m, aggregators.gars["median"](gradients=g))
assert tools.parse_keyval(["a:1", "b:x"]) == {"a": 1, "b": "x"}
assert callable(tools.pairwise) and hasattr(tools, "Context") and issubclass(tools.UserException, Exception)
assert callable(gtools.select_model) and callable(gtools.select_loss) and callable(gtools.select_optimizer)
net = gtools.select_model("convnet", torch.device("cpu"), "mnist")
assert sum(p.numel() for p in net.parameters()) == 21840
assert hasattr(datasets, "DatasetManager") and hasattr(datasets, "DataPartitioner")
assert issubclass(ByzWorker, Worker) and callable(Server)
print("compat ok")
'''


def test_reference_import_names_resolve_and_run():
    env = dict(os.environ, PYTHONPATH=f"{REPO}{os.pathsep}{REPO / 'compat'}", CUDA_VISIBLE_DEVICES="",
               GARFIELD_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, timeout=300, env=env,
                       cwd="/tmp")
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "compat ok" in r.stdout
