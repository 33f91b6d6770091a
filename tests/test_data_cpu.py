"""Datasets: the bundled PIMA rows (reference ``pima_diabetes.csv``) and the
reference's split / normalisation (``garfieldpp/datasets.py:52-94``)."""
import numpy as np
import torch

from garfield_amd.data.datasets import DataPartitioner, PimaDiabetesDataset


def test_pima_bundled_rows_and_reference_normalisation():
    tr, te = PimaDiabetesDataset(train=True), PimaDiabetesDataset(train=False)
    assert not tr.synthetic and len(tr) == 600 and len(te) == 168
    assert tr.x.shape == (600, 8) and tr.y.shape == (600, 1) and tr.x.dtype == torch.float32
    # each split normalised with its own mean / sample std (pandas semantics)
    for ds in (tr, te):
        assert torch.allclose(ds.x.mean(0), torch.zeros(8), atol=1e-5)
        assert torch.allclose(ds.x.std(0), torch.ones(8), atol=1e-4)
    # the public data set: 268 of 768 rows are positive; first row 6,148,72,35,0,33.6,0.627,50,1
    assert int(tr.y.sum() + te.y.sum()) == 268 - int(np.load(
        PimaDiabetesDataset.__init__.__globals__["PIMA_BUNDLED"])["rows"][600:-168, 8].sum())
    assert float(tr.y[0]) == 1.0


def test_pima_train_size_and_partitioner():
    tr = PimaDiabetesDataset(train=True, train_size=100)
    assert len(tr) == 100
    dp = DataPartitioner(list(range(10)), [0.5, 0.5])
    assert sorted(dp.partitions[0] + dp.partitions[1]) == list(range(10))
    assert sorted(list(dp.use(0)) + list(dp.use(1))) == list(range(10))
