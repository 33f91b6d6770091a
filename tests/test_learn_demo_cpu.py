"""LEARN web demo (reference LEARN/demo.py): the routes, input validation and one
real 3-node run (one epoch) through the HTTP API."""
import time

import pytest

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402

from garfield_amd.apps.learn_demo import Trainer, create_app  # noqa: E402


def test_routes_and_validation():
    client = TestClient(create_app(epochs=1))
    r = client.get("/")
    assert r.status_code == 200 and "LEARN" in r.text
    assert client.post("/", json={"n": 11, "f": 0}).status_code == 400
    assert client.post("/", json={"n": 3, "f": 0, "gar": "nope"}).status_code == 400
    assert client.get("/status", params={"trainer_id": 99}).status_code == 400
    with pytest.raises(ValueError):
        Trainer(3, 3, "median")


def test_demo_run_end_to_end():
    client = TestClient(create_app(epochs=1))
    r = client.post("/", json={"n": 3, "f": 1, "gar": "median"})
    assert r.status_code == 200
    tid = r.json()["trainerId"]
    deadline = time.time() + 240
    seen = []
    while time.time() < deadline:
        st = client.get("/status", params={"trainer_id": tid}).json()
        assert "error" not in st, st
        if "result" in st:
            break
        seen.append(st["progress"])
        time.sleep(0.5)
    assert "result" in st, seen
    assert 0.0 <= st["result"] <= 100.0
