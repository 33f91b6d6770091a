"""LEARN web demo: start a decentralised Byzantine-resilient training run from a
browser and watch its progress.

Reference: ``pytorch_impl/applications/LEARN/demo.py`` (Quart app, 453 lines) and
``templates/index.html`` (Vue page): ``GET /`` serves the page, ``POST /`` with
``{"n", "f", "gar"}`` starts ``n`` LEARN nodes (one process each, RPC on
localhost; ranks < f are Byzantine workers with the ``random`` attack) training
``pimanet`` on the PIMA diabetes data with RMSProp for 15 epochs and returns
``{"trainerId"}``; ``GET /status?trainer_id=`` answers ``{"progress": %}``, then
``{"result": mean final accuracy}`` or ``{"error"}``. A run that reports no
progress for 60 s is killed. Quart is not available offline, so the same routes
are served by FastAPI/uvicorn (``python -m garfield_amd.apps.learn_demo``);
``python -m garfield_amd.apps.learn_demo init_demo`` pre-loads the dataset and the
native extension like the reference's ``quart init_demo``.
"""

import argparse
import json
import math
import multiprocessing as mp
import queue
import socket
import threading

DATASET, MODEL, BATCH, EPOCHS = "pima", "pimanet", 16, 15
OPT_ARGS = {"lr": 0.001, "momentum": 0.9, "weight_decay": 0.0005}
NB_TRAIN = 600   # PIMA train split (reference datasets.py:52-94)

PAGE = """<!doctype html>
<html><head><meta charset="utf-8"><title>Garfield LEARN demo</title>
<style>body{font-family:sans-serif;max-width:40em;margin:2em auto}label{display:block;margin:.5em 0}
#bar{height:1.2em;background:#ddd}#fill{height:100%;width:0;background:#4a7}</style></head>
<body><h1>LEARN: decentralised Byzantine-resilient learning</h1>
<p>Each node is a worker and a parameter server; the first <i>f</i> nodes send random gradients.</p>
<label>Nodes n <input id="n" type="number" min="1" max="10" value="5"></label>
<label>Byzantine nodes f <input id="f" type="number" min="0" max="9" value="1"></label>
<label>Aggregation rule <select id="gar"><option>median</option><option>krum</option><option>average</option>
<option>trimmed-mean</option><option>bulyan</option><option>aksel</option><option>brute</option></select></label>
<button onclick="start()">Train</button>
<div id="bar"><div id="fill"></div></div><p id="msg"></p>
<script>
async function start(){
  const body={n:+document.getElementById('n').value,f:+document.getElementById('f').value,
              gar:document.getElementById('gar').value};
  const r=await fetch('/',{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify(body)});
  const j=await r.json(); if(j.error){msg(j.error);return;} poll(j.trainerId);}
function msg(t){document.getElementById('msg').textContent=t;}
async function poll(id){
  const j=await (await fetch('/status?trainer_id='+id)).json();
  if(j.error){msg('error: '+j.error);return;}
  if(j.result!==undefined){document.getElementById('fill').style.width='100%';
    msg('final accuracy: '+j.result.toFixed(2)+'%');return;}
  document.getElementById('fill').style.width=j.progress+'%';msg('training... '+j.progress+'%');
  setTimeout(()=>poll(id),1000);}
</script></body></html>
"""


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _node(rank: int, n: int, f: int, gar: str, port: int, num_iter: int, q) -> None:
    """One LEARN node (reference ``demo.py:89-241``), reporting progress on ``q``."""
    import os

    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from garfield_amd.apps import learn

    argv = ["--rank", str(rank), "--num_nodes", str(n), "--f", str(f), "--gar", gar, "--dataset", DATASET,
            "--model", MODEL, "--loss", "binary-cross-entropy", "--optimizer", "rmsprop", "--opt_args",
            json.dumps({k: str(v) for k, v in OPT_ARGS.items()}), "--batch", str(BATCH), "--num_iter",
            str(num_iter), "--acc_freq", "0", "--port", str(port), "--master", "127.0.0.1", "--device", "cpu",
            "--train_size", str(NB_TRAIN)]
    if rank < f:
        argv += ["--attack", "random"]
    res: dict = {}
    last = [-1]

    def progress(done, total):
        pct = done * 100 // total
        if pct != last[0]:
            last[0] = pct
            q.put({"rank": rank, "progress": pct})

    try:
        learn.main(argv, results=res, progress=progress)
        q.put({"rank": rank, "progress": 100, "result": float(res.get("accuracy") or 0.0)})
    except Exception as e:  # noqa: BLE001 - reported to the web client
        q.put({"rank": rank, "error": repr(e)})


class Trainer:
    """One demo run (reference ``demo.py:244-354``)."""

    TIMEOUT_PROGRESS_SEC = 60
    TIMEOUT_TERMINATE_SEC = 10

    def __init__(self, n: int, f: int, gar: str, port: int | None = None, epochs: int = EPOCHS):
        if n < 1 or n > 10:
            raise ValueError("The total number of nodes must be between 1 and 10")
        if f < 0 or f >= n:
            raise ValueError("The number of Byzantine nodes must be in [0, n)")
        from garfield_amd import aggregators

        if gar not in aggregators.gars:
            raise ValueError(f"unknown aggregation rule {gar!r}")
        self.n, self.f, self.gar = n, f, gar
        self.port = port or _free_port()
        self.num_iter = max(1, epochs * math.ceil(NB_TRAIN / (n * BATCH)))
        self.lock = threading.Lock()
        self.status = {r: 0 for r in range(n)}
        self.result: float | None = None
        self.error: str | None = None
        self.done = threading.Event()

    def train(self) -> None:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_node, args=(r, self.n, self.f, self.gar, self.port, self.num_iter, q),
                             daemon=True) for r in range(self.n)]
        for p in procs:
            p.start()
        accs = []
        try:
            while len(accs) < self.n:
                msg = q.get(timeout=self.TIMEOUT_PROGRESS_SEC)
                if "error" in msg:
                    raise RuntimeError(f"node {msg['rank']}: {msg['error']}")
                with self.lock:
                    self.status[msg["rank"]] = msg["progress"]
                if "result" in msg:
                    accs.append(msg["result"])
            with self.lock:
                self.result = sum(accs) / len(accs)
        except (queue.Empty, RuntimeError) as e:
            with self.lock:
                self.error = "Timeout while waiting for progress" if isinstance(e, queue.Empty) else str(e)
            for p in procs:
                p.kill()
        finally:
            for p in procs:
                p.join(timeout=self.TIMEOUT_TERMINATE_SEC)
                if p.is_alive():
                    p.kill()
            self.done.set()

    def run(self) -> None:
        threading.Thread(target=self.train, daemon=True).start()

    def get_status(self) -> dict:
        with self.lock:
            if self.error is not None:
                return {"error": self.error}
            if self.result is not None:
                return {"result": self.result}
            return {"progress": sum(self.status.values()) // len(self.status)}


class Trainers:
    def __init__(self):
        self.lock = threading.Lock()
        self.trainers: dict[int, Trainer] = {}
        self.next_id = 0

    def submit(self, trainer: Trainer) -> int:
        with self.lock:
            tid = self.next_id
            self.next_id += 1
            self.trainers[tid] = trainer
        trainer.run()
        return tid

    def get_status(self, tid: int) -> dict:
        with self.lock:
            t = self.trainers.get(tid)
        if t is None:
            raise ValueError(f"Trainer ID {tid} does not exist")
        return t.get_status()


def create_app(epochs: int = EPOCHS):
    from fastapi import FastAPI, Request
    from fastapi.responses import HTMLResponse, JSONResponse

    app = FastAPI(title="Garfield LEARN demo")
    trainers = Trainers()
    app.state.trainers = trainers

    @app.get("/", response_class=HTMLResponse)
    async def index():
        return PAGE

    @app.post("/")
    async def train(request: Request):
        try:
            form = await request.json()
            t = Trainer(int(form["n"]), int(form["f"]), form.get("gar", "average"),
                        epochs=int(form.get("epochs", epochs)))
            return {"trainerId": trainers.submit(t)}
        except Exception as e:  # noqa: BLE001
            return JSONResponse({"error": str(e)}, status_code=400)

    @app.get("/status")
    async def status(trainer_id: int):
        try:
            return trainers.get_status(trainer_id)
        except Exception as e:  # noqa: BLE001
            return JSONResponse({"error": str(e)}, status_code=400)

    return app


def init_demo() -> None:
    """Pre-load the PIMA data and the native extension (reference ``quart init_demo``)."""
    from garfield_amd import _native
    from garfield_amd.data.datasets import fetch

    fetch(DATASET, train=True)
    _native.available()


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("command", nargs="?", default="serve", choices=["serve", "init_demo"])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--epochs", type=int, default=EPOCHS)
    a = ap.parse_args(argv)
    if a.command == "init_demo":
        init_demo()
        return
    import uvicorn

    uvicorn.run(create_app(a.epochs), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
