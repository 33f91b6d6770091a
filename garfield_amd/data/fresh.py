"""Fresh, augmented training batches built on the GPU in one launch per step.

The reference trains every worker from a host DataLoader over CIFAR-10 with
RandomCrop(32, padding=4) + RandomHorizontalFlip + Normalize
(``pytorch_impl/libs/garfieldpp/datasets.py:99-140``). ``DeviceBatches`` keeps the
(uint8, NHWC) images of a dataset resident in HBM and, per step, draws the k
logical workers' sample indices on the device and builds the whole grouped batch
with ``data_aug.hip`` (gather + random crop + flip + normalise + bf16 cast,
channels_last; fp32 when the consumer's step runs at the reference precision) — no host work, no
per-image launches. The crop/flip of a row is a
hash of (seed, step, row), so a step's batch is reproducible.

CPU tensors take a PyTorch implementation of the same augmentation (same hash is
not reproduced bit-for-bit; the CPU path is for tests and small runs).
"""
from __future__ import annotations

import torch

from garfield_amd import _native

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)


class DeviceBatches:
    """``next()`` -> list of k (x, y) micro-batches of B rows each (views into one grouped
    buffer that is rewritten every step), drawn with replacement from ``images``."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, k: int, batch: int, device,
                 mean=CIFAR_MEAN, std=CIFAR_STD, pad: int = 4, flip: bool = True, seed: int = 0):
        if images.dtype != torch.uint8 or images.dim() != 4:
            raise ValueError("images must be a uint8 [N, H, W, C] tensor")
        self.device = torch.device(device)
        self.src = images.to(self.device).contiguous()
        self.labels = labels.to(self.device).long()
        n, h, w, c = self.src.shape
        if len(mean) != c or len(std) != c:
            raise ValueError("one mean / std per channel")
        self.k, self.B = int(k), int(batch)
        self.mean, self.std = [float(m) for m in mean], [float(s) for s in std]
        self.pad, self.flip, self.seed = int(pad), bool(flip), int(seed)
        self.step = 0
        R = self.k * self.B
        if self.device.type == "cuda":   # the kernel writes bf16 NHWC rows: the grouped step's input layout
            self.out = torch.empty((R, c, h, w), dtype=torch.bfloat16, device=self.device,
                                   memory_format=torch.channels_last)
        else:
            self.out = torch.empty((R, c, h, w), dtype=torch.float32)
        self.lab_out = torch.empty(R, dtype=torch.long, device=self.device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(self.seed)

    def attach(self, buffers) -> bool:
        """Write every batch straight into a consumer's input buffers (x [k*B, C, H, W] bf16 or fp32
        channels_last, y [k*B] int64: ``RobustDataParallel.grouped_inputs``); False (nothing
        changed) when they do not fit."""
        if buffers is None or self.device.type != "cuda":
            return False
        x, y = buffers
        if (tuple(x.shape) != tuple(self.out.shape) or x.dtype not in (torch.bfloat16, torch.float32)
                or x.device != self.device
                or not x.is_contiguous(memory_format=torch.channels_last) or y.dtype != torch.long
                or tuple(y.shape) != (self.k * self.B,) or not y.is_contiguous()):
            return False
        self.out, self.lab_out = x, y
        return True

    @classmethod
    def synthetic(cls, num_images: int, shape, num_classes: int, k: int, batch: int, device, seed: int = 0,
                  learnable: bool = True, **kw):
        """A random uint8 dataset of ``num_images`` images of ``shape`` (C, H, W).

        ``learnable``: each class has a fixed random base colour (shared by every rank and
        seed) and an image is its class colour plus uniform per-pixel noise of +-64, so the
        label survives the crop (black padding) and the flip and training makes visible
        progress (the loss falls below ln(num_classes)); else the labels are random."""
        g = torch.Generator().manual_seed(seed)
        c, h, w = shape
        labels = torch.randint(0, num_classes, (num_images,), generator=g)
        if learnable:
            colours = torch.randint(64, 192, (num_classes, c), generator=torch.Generator().manual_seed(424242))
            noise = torch.randint(-64, 65, (num_images, h, w, c), generator=g)
            imgs = (colours[labels][:, None, None, :] + noise).clamp_(0, 255).to(torch.uint8)
        else:
            imgs = torch.randint(0, 256, (num_images, h, w, c), dtype=torch.uint8, generator=g)
        mean = kw.pop("mean", CIFAR_MEAN if c == 3 else (0.5,) * c)
        std = kw.pop("std", CIFAR_STD if c == 3 else (0.25,) * c)
        return cls(imgs, labels, k, batch, device, mean=mean, std=std, seed=seed, **kw)

    def next(self):
        R = self.k * self.B
        if self.device.type == "cuda":
            # ONE launch: sample indices (hash), gather + crop + flip + normalise, labels
            _native.native().gpu_augment_gather(self.src, None, self.seed, self.step, self.mean, self.std, self.out,
                                                self.pad, self.flip, self.labels, self.lab_out)
            torch.autograd.graph.increment_version(self.out)   # written by a native kernel: consumers see a new version
            torch.autograd.graph.increment_version(self.lab_out)
            y = self.lab_out
        else:
            idx = torch.randint(0, self.src.shape[0], (R,), generator=self.gen, device=self.device)
            self.out.copy_(self._cpu(idx))
            y = self.labels[idx]
        self.step += 1
        return [(self.out[j * self.B:(j + 1) * self.B], y[j * self.B:(j + 1) * self.B]) for j in range(self.k)]

    def _cpu(self, idx: torch.Tensor) -> torch.Tensor:
        x = self.src[idx].permute(0, 3, 1, 2).float().div_(255.0)
        m = torch.tensor(self.mean).view(1, -1, 1, 1)
        s = torch.tensor(self.std).view(1, -1, 1, 1)
        R, c, h, w = x.shape
        p = self.pad
        if p:
            x = torch.nn.functional.pad(x, (p, p, p, p))
            oy = torch.randint(0, 2 * p + 1, (R,), generator=self.gen)
            ox = torch.randint(0, 2 * p + 1, (R,), generator=self.gen)
            x = torch.stack([x[i, :, oy[i]:oy[i] + h, ox[i]:ox[i] + w] for i in range(R)])
        if self.flip:
            fl = torch.rand(R, generator=self.gen) < 0.5
            x = torch.where(fl[:, None, None, None], x.flip(3), x)
        return (x - m) / s
