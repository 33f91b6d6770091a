"""Datasets, per-worker partitioning and device-resident batch pipelines.

Reference: ``pytorch_impl/libs/garfieldpp/datasets.py:47-250`` (torchvision MNIST /
CIFAR-10 with augmentation, PIMA csv, ``Partition``, ``DataPartitioner(sizes,
seed=1234)``, ``DatasetManager``; ``get_train_set`` materialises the whole
partition as a Python list of batches with the augmentation sampled ONCE).

Here (no torchvision, no network):

* MNIST is read from the raw IDX files and CIFAR-10 from the *binary* batches
  (``cifar-10-batches-bin``) under ``$GARFIELD_DATA`` or ``~/data`` — no pickle;
  when the files are absent a deterministic synthetic dataset of the same shape is
  used (and reported), so every app runs offline;
* ``DeviceLoader`` keeps a whole partition resident on the GPU (CIFAR-10 is 150 MB
  of uint8; HBM is 288 GB) and draws fresh augmentations (random crop with
  4-pixel padding + horizontal flip + normalisation) on the device every epoch.
"""
from __future__ import annotations

import functools
import gzip
import os
import pathlib
from random import Random

import numpy as np
import torch

from garfield_amd.utils.logging import warning

datasets_list = ["mnist", "cifar10", "cifar100", "pima", "synthetic", "imagenet"]

MNIST_MEAN, MNIST_STD = (0.1307,), (0.3081,)
CIFAR_MEAN, CIFAR_STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)  # reference datasets.py:196

SHAPES = {"mnist": (1, 28, 28), "cifar10": (3, 32, 32), "cifar100": (3, 32, 32), "pima": (8,),
          "synthetic": (3, 32, 32), "imagenet": (3, 224, 224)}
CLASSES = {"mnist": 10, "cifar10": 10, "cifar100": 100, "pima": 1, "synthetic": 10, "imagenet": 1000}
SIZES = {"mnist": (60000, 10000), "cifar10": (50000, 10000), "cifar100": (50000, 10000), "pima": (600, 168),
         "synthetic": (50000, 10000), "imagenet": (12800, 500)}


def data_root() -> pathlib.Path:
    return pathlib.Path(os.environ.get("GARFIELD_DATA", str(pathlib.Path.home() / "data")))


class TensorDataset(torch.utils.data.Dataset):
    """(inputs, targets) held as tensors; ``inputs`` may be uint8 images (normalised on access)."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor, mean=None, std=None, name: str = "", synthetic=False):
        self.x, self.y = x, y
        self.mean = None if mean is None else torch.tensor(mean).view(-1, 1, 1)
        self.std = None if std is None else torch.tensor(std).view(-1, 1, 1)
        self.name = name
        self.synthetic = synthetic

    def __len__(self):
        return self.x.shape[0]

    def _norm(self, x):
        if x.dtype == torch.uint8:
            x = x.float() / 255.0
            if self.mean is not None:
                x = (x - self.mean) / self.std
        return x

    def __getitem__(self, i):
        return self._norm(self.x[i]), self.y[i]


def _read_idx(path: pathlib.Path) -> np.ndarray:
    opener = gzip.open if path.suffix == ".gz" else open
    with opener(path, "rb") as fh:
        data = fh.read()
    ndim = data[3]
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def _find(*cands) -> pathlib.Path | None:
    for c in cands:
        for p in (c, c.with_name(c.name + ".gz")):
            if p.exists():
                return p
    return None


def _synthetic(name: str, train: bool, n: int | None = None, seed: int = 0) -> TensorDataset:
    shape, k = SHAPES[name], max(CLASSES[name], 2)
    n = n or SIZES[name][0 if train else 1]
    g = torch.Generator().manual_seed(seed + (0 if train else 1))
    proj = torch.randn(int(np.prod(shape)), k, generator=torch.Generator().manual_seed(4242))
    x = torch.randn((n, *shape), generator=g)
    logits = x.flatten(1) @ proj
    if CLASSES[name] == 1:
        y = (logits[:, 0] > 0).float().unsqueeze(1)
    else:
        y = logits.argmax(1)
    return TensorDataset(x, y, name=name, synthetic=True)


def load_mnist(train: bool) -> TensorDataset:
    root = data_root()
    stem = "train" if train else "t10k"
    xi = _find(root / "MNIST" / "raw" / f"{stem}-images-idx3-ubyte", root / f"{stem}-images-idx3-ubyte")
    yi = _find(root / "MNIST" / "raw" / f"{stem}-labels-idx1-ubyte", root / f"{stem}-labels-idx1-ubyte")
    if xi is None or yi is None:
        warning(f"MNIST not found under {root}; using a synthetic MNIST-shape dataset")
        return _synthetic("mnist", train)
    x = torch.from_numpy(_read_idx(xi).copy()).unsqueeze(1)
    y = torch.from_numpy(_read_idx(yi).astype(np.int64))
    return TensorDataset(x, y, MNIST_MEAN, MNIST_STD, "mnist")


def load_cifar10(train: bool) -> TensorDataset:
    root = data_root() / "cifar-10-batches-bin"
    files = [root / f"data_batch_{i}.bin" for i in range(1, 6)] if train else [root / "test_batch.bin"]
    if not all(f.exists() for f in files):
        warning(f"CIFAR-10 binary batches not found under {root}; using a synthetic CIFAR-10-shape dataset")
        return _synthetic("cifar10", train)
    raw = np.concatenate([np.fromfile(f, dtype=np.uint8).reshape(-1, 3073) for f in files])
    y = torch.from_numpy(raw[:, 0].astype(np.int64))
    x = torch.from_numpy(raw[:, 1:].reshape(-1, 3, 32, 32).copy())
    return TensorDataset(x, y, CIFAR_MEAN, CIFAR_STD, "cifar10")


PIMA_BUNDLED = pathlib.Path(__file__).with_name("pima_diabetes.npz")


class PimaDiabetesDataset(TensorDataset):
    """PIMA Indians diabetes (8 features, binary outcome): the first 600 rows train, the
    last 168 test, each split z-normalised with its OWN mean and sample standard
    deviation (reference datasets.py:52-94, pandas ``std``).

    Source, first found: ``csv`` / ``$GARFIELD_PIMA_CSV`` (the reference's CSV layout),
    then the bundled ``pima_diabetes.npz`` (the same 768 rows as the reference's
    ``pima_diabetes.csv``, the public UCI/NIDDK Pima Indians Diabetes data, stored as a
    float32 array; loaded with ``allow_pickle=False``), else synthetic rows of the same
    shape (with a warning)."""

    TRAIN_SPLIT, TEST_SPLIT = 600, 168

    def __init__(self, train: bool = True, train_size: int | None = None, csv: str | None = None):
        path = csv or os.environ.get("GARFIELD_PIMA_CSV")
        arr = None
        if path and pathlib.Path(path).exists():
            arr = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.float64)
        elif PIMA_BUNDLED.exists():
            with np.load(PIMA_BUNDLED, allow_pickle=False) as z:
                arr = z["rows"].astype(np.float64)
        ntrain = min(train_size or self.TRAIN_SPLIT, self.TRAIN_SPLIT)
        if arr is None:
            warning("PIMA data not found; using synthetic PIMA-shape rows")
            s = _synthetic("pima", train, n=ntrain if train else self.TEST_SPLIT)
            super().__init__(s.x, s.y, name="pima", synthetic=True)
            return
        rows = arr[:ntrain] if train else arr[-self.TEST_SPLIT:]
        feats, lab = rows[:, :8], rows[:, 8:9]
        feats = (feats - feats.mean(0)) / feats.std(0, ddof=1)
        super().__init__(torch.from_numpy(feats.astype(np.float32)), torch.from_numpy(lab.astype(np.float32)),
                         name="pima")


@functools.lru_cache(maxsize=8)
def fetch(name: str, train: bool = True, train_size: int | None = None) -> TensorDataset:
    if name not in datasets_list:
        raise ValueError(f"Existing datasets are: {datasets_list}")
    if name == "mnist":
        return load_mnist(train)
    if name == "cifar10":
        return load_cifar10(train)
    if name == "pima":
        return PimaDiabetesDataset(train=train, train_size=train_size)
    return _synthetic(name, train)


class Partition(torch.utils.data.Dataset):
    """Dataset view restricted to ``index`` (reference datasets.py:97-118)."""

    def __init__(self, data, index):
        self.data = data
        self.index = index

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        return self.data[self.index[i]]


class DataPartitioner:
    """Split a dataset into consecutive chunks of the given fractions, each shuffled
    with a seeded RNG (reference datasets.py:121-150)."""

    def __init__(self, data, sizes=(0.7, 0.2, 0.1), seed: int = 1234):
        self.data = data
        self.partitions = []
        rng = Random(seed)
        indexes = list(range(len(data)))
        for frac in sizes:
            n = int(frac * len(data))
            part, indexes = indexes[:n], indexes[n:]
            rng.shuffle(part)
            self.partitions.append(part)

    def use(self, partition: int) -> Partition:
        return Partition(self.data, self.partitions[partition])


class DeviceLoader:
    """A partition resident on ``device``; yields (x, y) batches with on-device
    augmentation. Indexable like the reference's materialised batch list
    (``loader[i % len(loader)]``), but draws a fresh augmentation per epoch."""

    def __init__(self, ds: TensorDataset, index, batch: int, device, augment: bool = False, shuffle: bool = False,
                 seed: int = 0, drop_last: bool = False):
        idx = torch.as_tensor(list(index), dtype=torch.long)
        self.x = ds.x[idx].to(device)
        self.y = ds.y[idx].to(device)
        self.mean = None if ds.mean is None else ds.mean.to(device)
        self.std = None if ds.std is None else ds.std.to(device)
        self.batch = batch
        self.augment = augment and self.x.dim() == 4
        self.shuffle = shuffle
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.drop_last = drop_last
        self._epoch_order = None
        self._epoch = -1

    def __len__(self):
        n = self.x.shape[0]
        return n // self.batch if self.drop_last else (n + self.batch - 1) // self.batch

    def _order(self, epoch: int):
        if not self.shuffle:
            return None
        if epoch != self._epoch:
            self._epoch_order = torch.randperm(self.x.shape[0], generator=self.gen, device=self.device)
            self._epoch = epoch
        return self._epoch_order

    def _prep(self, x: torch.Tensor) -> torch.Tensor:
        if x.dtype == torch.uint8:
            x = x.float().div_(255.0)
            if self.mean is not None:
                x = (x - self.mean) / self.std
        if self.augment:
            b, c, h, w = x.shape
            pad = torch.nn.functional.pad(x, (4, 4, 4, 4))
            ox = torch.randint(0, 9, (b,), generator=self.gen, device=self.device)
            oy = torch.randint(0, 9, (b,), generator=self.gen, device=self.device)
            ar = torch.arange(h, device=self.device)
            rows = (oy[:, None] + ar[None, :])[:, None, :, None].expand(b, c, h, w + 8)
            pad = torch.gather(pad, 2, rows)
            cols = (ox[:, None] + ar[None, :])[:, None, None, :].expand(b, c, h, w)
            x = torch.gather(pad, 3, cols)
            flip = torch.rand(b, generator=self.gen, device=self.device) < 0.5
            x = torch.where(flip[:, None, None, None], x.flip(3), x)
        return x

    def __getitem__(self, i: int):
        nb = len(self)
        epoch, j = divmod(i, nb)
        order = self._order(epoch)
        lo, hi = j * self.batch, min((j + 1) * self.batch, self.x.shape[0])
        sel = slice(lo, hi) if order is None else order[lo:hi]
        return self._prep(self.x[sel]), self.y[sel]

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


class DatasetManager:
    """Train/test sets of one node (reference datasets.py:152-250): ``minibatch`` per
    worker, the train set split in ``num_workers`` equal partitions, partition
    ``rank - num_ps`` for this node (``size`` = total nodes)."""

    def __init__(self, dataset, minibatch, num_workers, size, rank, train_size=None, device=None):
        if dataset not in datasets_list:
            raise ValueError(f"Existing datasets are: {datasets_list}")
        self.dataset = dataset
        self.batch = minibatch * num_workers
        self.num_workers = num_workers
        self.num_ps = size - num_workers
        self.rank = rank
        self.train_size = train_size
        self.device = device or ("cuda" if torch.cuda.is_available() else "cpu")

    def fetch_dataset(self, train=True):
        return fetch(self.dataset, train, self.train_size)

    def get_train_set(self) -> DeviceLoader:
        ds = self.fetch_dataset(train=True)
        size = self.num_workers
        bsz = int(self.batch / float(size))
        part = DataPartitioner(ds, [1.0 / size] * size).partitions[max(self.rank - self.num_ps, 0) % size]
        return DeviceLoader(ds, part, bsz, self.device, augment=self.dataset in ("cifar10", "cifar100"),
                            seed=1234 + self.rank)

    def get_test_set(self) -> DeviceLoader:
        ds = self.fetch_dataset(train=False)
        return DeviceLoader(ds, range(len(ds)), 100, self.device)


def poison_batch(x: torch.Tensor, y: torch.Tensor, severity: int, generator: torch.Generator | None = None):
    """Malformed-input (data poisoning) attack of the legacy ``mnistAttack`` experiment
    (``tensorflow_impl/applications/Garfield_legacy/experiments/mnistAttack.py:34-80``):
    severity 1 scales the inputs by -100; severity 2 scales them by -1e12 and
    shuffles the labels against the inputs. Severity 0 returns the batch unchanged."""
    if severity <= 0:
        return x, y
    if severity == 1:
        return x * -100.0, y
    perm = torch.randperm(y.shape[0], generator=generator, device="cpu").to(y.device)
    return x * -1e12, y[perm]
