"""Inception v3 (Szegedy et al., "Rethinking the Inception Architecture", 2016).

The TF reference builds ``tf.keras.applications.InceptionV3()`` for its "Inception"
model name (``tensorflow_impl/libs/model.py:59``); torchvision is not available in
this image, so the network is defined here from the paper's module table
(stem → 3×A(35×35) → B(grid reduction) → 4×C(17×17, factorised 7×7) → D(reduction)
→ 2×E(8×8, expanded filter banks) → pool → fc). Every conv is conv+BN+ReLU, which
MIOpen fuses on gfx950. Input 299×299 (ImageNet shape); any size ≥ 75 works since the
head uses adaptive pooling. No auxiliary classifier (it only adds a training-time
loss term that the Garfield trainers never use).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class ConvBN(nn.Sequential):
    def __init__(self, cin, cout, kernel, stride=1, padding=0):
        super().__init__(nn.Conv2d(cin, cout, kernel, stride=stride, padding=padding, bias=False),
                         nn.BatchNorm2d(cout, eps=1e-3), nn.ReLU(inplace=True))


class MixedA(nn.Module):
    """35×35 module: 1×1 | 1×1→5×5 | 1×1→3×3→3×3 | avgpool→1×1."""

    def __init__(self, cin, pool_features):
        super().__init__()
        self.b1 = ConvBN(cin, 64, 1)
        self.b5 = nn.Sequential(ConvBN(cin, 48, 1), ConvBN(48, 64, 5, padding=2))
        self.b3 = nn.Sequential(ConvBN(cin, 64, 1), ConvBN(64, 96, 3, padding=1), ConvBN(96, 96, 3, padding=1))
        self.bp = ConvBN(cin, pool_features, 1)

    def forward(self, x):
        p = F.avg_pool2d(x, 3, stride=1, padding=1)
        return torch.cat([self.b1(x), self.b5(x), self.b3(x), self.bp(p)], 1)


class ReductionB(nn.Module):
    """35×35 → 17×17: stride-2 3×3 | 1×1→3×3→3×3 (s2) | maxpool."""

    def __init__(self, cin):
        super().__init__()
        self.b3 = ConvBN(cin, 384, 3, stride=2)
        self.b33 = nn.Sequential(ConvBN(cin, 64, 1), ConvBN(64, 96, 3, padding=1), ConvBN(96, 96, 3, stride=2))

    def forward(self, x):
        return torch.cat([self.b3(x), self.b33(x), F.max_pool2d(x, 3, stride=2)], 1)


class MixedC(nn.Module):
    """17×17 module with factorised 7×7 convolutions (1×7 then 7×1)."""

    def __init__(self, cin, c7):
        super().__init__()
        self.b1 = ConvBN(cin, 192, 1)
        self.b7 = nn.Sequential(ConvBN(cin, c7, 1), ConvBN(c7, c7, (1, 7), padding=(0, 3)),
                                ConvBN(c7, 192, (7, 1), padding=(3, 0)))
        self.b77 = nn.Sequential(ConvBN(cin, c7, 1), ConvBN(c7, c7, (7, 1), padding=(3, 0)),
                                 ConvBN(c7, c7, (1, 7), padding=(0, 3)), ConvBN(c7, c7, (7, 1), padding=(3, 0)),
                                 ConvBN(c7, 192, (1, 7), padding=(0, 3)))
        self.bp = ConvBN(cin, 192, 1)

    def forward(self, x):
        p = F.avg_pool2d(x, 3, stride=1, padding=1)
        return torch.cat([self.b1(x), self.b7(x), self.b77(x), self.bp(p)], 1)


class ReductionD(nn.Module):
    """17×17 → 8×8."""

    def __init__(self, cin):
        super().__init__()
        self.b3 = nn.Sequential(ConvBN(cin, 192, 1), ConvBN(192, 320, 3, stride=2))
        self.b7 = nn.Sequential(ConvBN(cin, 192, 1), ConvBN(192, 192, (1, 7), padding=(0, 3)),
                                ConvBN(192, 192, (7, 1), padding=(3, 0)), ConvBN(192, 192, 3, stride=2))

    def forward(self, x):
        return torch.cat([self.b3(x), self.b7(x), F.max_pool2d(x, 3, stride=2)], 1)


class MixedE(nn.Module):
    """8×8 module with expanded filter banks (1×3 and 3×1 in parallel)."""

    def __init__(self, cin):
        super().__init__()
        self.b1 = ConvBN(cin, 320, 1)
        self.b3 = ConvBN(cin, 384, 1)
        self.b3a = ConvBN(384, 384, (1, 3), padding=(0, 1))
        self.b3b = ConvBN(384, 384, (3, 1), padding=(1, 0))
        self.bd = nn.Sequential(ConvBN(cin, 448, 1), ConvBN(448, 384, 3, padding=1))
        self.bda = ConvBN(384, 384, (1, 3), padding=(0, 1))
        self.bdb = ConvBN(384, 384, (3, 1), padding=(1, 0))
        self.bp = ConvBN(cin, 192, 1)

    def forward(self, x):
        y3 = self.b3(x)
        yd = self.bd(x)
        p = F.avg_pool2d(x, 3, stride=1, padding=1)
        return torch.cat([self.b1(x), self.b3a(y3), self.b3b(y3), self.bda(yd), self.bdb(yd), self.bp(p)], 1)


class InceptionV3(nn.Module):
    def __init__(self, num_classes: int = 1000, dropout: float = 0.5):
        super().__init__()
        self.stem = nn.Sequential(
            ConvBN(3, 32, 3, stride=2), ConvBN(32, 32, 3), ConvBN(32, 64, 3, padding=1), nn.MaxPool2d(3, 2),
            ConvBN(64, 80, 1), ConvBN(80, 192, 3), nn.MaxPool2d(3, 2))
        self.blocks = nn.Sequential(
            MixedA(192, 32), MixedA(256, 64), MixedA(288, 64), ReductionB(288),
            MixedC(768, 128), MixedC(768, 160), MixedC(768, 160), MixedC(768, 192), ReductionD(768),
            MixedE(1280), MixedE(2048))
        self.dropout = nn.Dropout(dropout)
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.fc(self.dropout(x))
