"""Reference ``tools`` helpers (PT libs/tools, TF rsrcs/tools) and the Checkpoints manager."""
import sys

import torch
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches
from garfield_amd.utils.checkpoint import Checkpoints
from garfield_amd.utils.misc import ExpandPath, device_from_tuple, make_interface, print_args


def test_checkpoints_keep_and_resume(tmp_path):
    torch.manual_seed(0)
    cfg = EngineConfig(gar="krum", f=1, workers_per_rank=5, lr=0.05)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(), cfg)
    b = synthetic_batches(5, 8, (1, 28, 28), 10, "cpu")
    ck = Checkpoints(str(tmp_path / "ck"), max_to_keep=2)
    for _ in range(3):
        eng.step(b)
        ck.save(eng)
    assert ck.steps() == [2, 3]
    ref = eng.flat_model().clone()
    eng.step(b)
    torch.manual_seed(0)
    eng2 = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(), cfg)
    ck.restore(eng2)
    assert eng2.step_count == 3 and torch.equal(eng2.flat_model(), ref)
    eng2.step(b)
    assert torch.allclose(eng2.flat_model(), eng.flat_model(), atol=1e-6)


def test_misc_helpers(capsys, tmp_path):
    print_args("rule", "krum", ["m:3"])
    assert "Selected rule: krum" in capsys.readouterr().out
    with ExpandPath(tmp_path):
        assert str(tmp_path) in sys.path
    assert str(tmp_path) not in sys.path
    freed = []
    Box = make_interface(lambda v: [v], lambda h: freed.append(h), get=lambda h: h[0], put=lambda h, v: h.__setitem__(0, v))
    b = Box(3)
    b.put(5)
    assert b.get() == 5 and b() == [5]
    del b
    assert freed == [[5]]
    assert device_from_tuple("ps", 1, "gpu", 0) == "/job:ps/replica:0/task:1/device:GPU:0"


def test_tf_flatten_helpers_roundtrip():
    import numpy as np
    import torch.nn as nn

    from garfield_amd.utils.flat import flatten_pairs, flatten_weights, inflate, mapflat, reshape_weights

    m = nn.Sequential(nn.Linear(3, 4), nn.Linear(4, 2))
    ps = list(m.parameters())
    grads = [torch.randn_like(p) for p in ps]
    pairs = list(zip(grads, ps)) + [(None, torch.zeros(1))]
    flat, fmap = flatten_pairs(pairs)
    assert flat.numel() == sum(p.numel() for p in ps)
    assert torch.equal(flatten_pairs(list(reversed(pairs)), fmap), flat)   # positions follow the map
    order = mapflat(fmap, ps)
    assert order == ps
    for (view, v), g in zip(inflate(flat, order), grads):
        assert view.shape == v.shape and torch.equal(view, g)
    w = flatten_weights(ps)
    assert isinstance(w, np.ndarray) and w.size == flat.numel()
    back = reshape_weights(m, w)
    for a, p in zip(back, ps):
        np.testing.assert_array_equal(a, p.detach().numpy())


def test_trace_graph_prints_begin_end(capsys):
    from garfield_amd.utils.profiling import trace_graph

    f = trace_graph(lambda a, b: a + b, "add")
    assert f(2, 3) == 5
    out = capsys.readouterr().out
    assert "[TRACE] (begin) add" in out and "[TRACE] (end)   add" in out


def test_checkpoint_channels_last_to_nchw_roundtrip(tmp_path):
    """Momentum is saved in the reference layout: a checkpoint of a grouped
    (channels_last memory order) engine resumes an NCHW engine exactly."""
    from garfield_amd.utils.checkpoint import load_engine, save_engine

    kw = dict(gar="krum", f=1, workers_per_rank=5, lr=0.05, autocast_dtype=None, exchange_dtype=torch.float32)
    torch.manual_seed(0)
    a = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(),
                           EngineConfig(worker_batching=True, **kw))
    assert a._gexec is not None
    conv = next(p for p in a.model.parameters() if p.dim() == 4)
    assert conv.is_contiguous(memory_format=torch.channels_last) and not conv.is_contiguous()
    b = synthetic_batches(5, 2, (3, 32, 32), 10, "cpu")
    for _ in range(2):
        a.step(b)
    save_engine(str(tmp_path / "a.pt"), a)
    torch.manual_seed(1)
    c = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(),
                           EngineConfig(worker_batching=False, **kw))
    assert c._gexec is None
    load_engine(str(tmp_path / "a.pt"), c)
    assert torch.equal(c.flat.reference_vector(), a.flat.reference_vector())
    assert torch.equal(c.flat.to_reference(c.mom), a.flat.to_reference(a.mom))
    a.step(b)
    c.step(b)
    ra, rc = a.flat.reference_vector(), c.flat.reference_vector()
    assert ((ra - rc).norm() / ra.norm()).item() < 1e-5


def test_checkpoint_without_layout_key_is_reference_layout(tmp_path):
    """Checkpoints written before the ``momentum_layout`` key existed already held the momentum
    in the reference layout: loading one into a channels_last (grouped) engine must reorder it."""
    from garfield_amd.utils.checkpoint import load_engine, save_engine

    kw = dict(gar="krum", f=1, workers_per_rank=5, lr=0.05, autocast_dtype=None, exchange_dtype=torch.float32)
    torch.manual_seed(0)
    a = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(),
                           EngineConfig(worker_batching=True, **kw))
    b = synthetic_batches(5, 2, (3, 32, 32), 10, "cpu")
    a.step(b)
    p = str(tmp_path / "a.pt")
    save_engine(p, a)
    state = torch.load(p, weights_only=True)
    del state["momentum_layout"]                    # the format of the earlier revision
    torch.save(state, p)
    torch.manual_seed(1)
    c = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(),
                           EngineConfig(worker_batching=True, **kw))
    assert not torch.equal(a.flat.to_reference(a.mom), a.mom)   # memory order differs from reference order
    load_engine(p, c)
    assert torch.equal(c.mom, a.mom)
    assert torch.equal(c.flat.to_reference(c.mom), a.flat.to_reference(a.mom))
