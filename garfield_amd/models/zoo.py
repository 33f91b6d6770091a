"""CIFAR-scale model families of the reference's ``select_model`` list
(``garfieldpp/tools.py:66-88``; reference implementations in ``garfieldpp/models/*.py``,
the pytorch-cifar family): PreActResNet, GoogLeNet, DenseNet, ResNeXt29, MobileNet,
MobileNetV2, DPN, ShuffleNet (v1 g2/g3, v2), SENet18, EfficientNetB0, RegNetX,
PNASNet and CIFAR VGG; plus the torchvision ImageNet VGG16/19 the reference builds
for ``vgg16`` / ``vgg19``. Written from the published architectures; every model
takes ``num_classes`` and NCHW input (32x32 for the CIFAR families).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def conv_bn(cin, cout, k=3, s=1, p=None, groups=1, act=True):
    p = (k - 1) // 2 if p is None else p
    layers = [nn.Conv2d(cin, cout, k, s, p, groups=groups, bias=False), nn.BatchNorm2d(cout)]
    if act:
        layers.append(nn.ReLU(inplace=True))
    return nn.Sequential(*layers)


# ------------------------------------------------------------------ PreActResNet

class PreActBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(cin)
        self.conv1 = nn.Conv2d(cin, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.shortcut = None
        if stride != 1 or cin != planes:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, planes, 1, stride, bias=False))

    def forward(self, x):
        out = F.relu(self.bn1(x))
        sc = self.shortcut(out) if self.shortcut is not None else x
        out = self.conv1(out)
        out = self.conv2(F.relu(self.bn2(out)))
        return out + sc


class PreActResNet(nn.Module):
    """Pre-activation ResNet (He et al. 2016): no BatchNorm after the last block, as in
    the reference ``models/preact_resnet.py`` (same parameter list, so its flat
    vectors load here)."""

    def __init__(self, block, blocks, num_classes=10, stem_bn=False):
        super().__init__()
        self.cin = 64
        self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64) if stem_bn else None   # SENet's stem
        for i, (w, n, s) in enumerate(zip((64, 128, 256, 512), blocks, (1, 2, 2, 2))):
            setattr(self, f"layer{i + 1}", self._make(block, w, n, s))
        self.linear = nn.Linear(512 * block.expansion, num_classes)

    def _make(self, block, planes, n, stride):
        mods = []
        for s in [stride] + [1] * (n - 1):
            mods.append(block(self.cin, planes, s))
            self.cin = planes * block.expansion
        return nn.Sequential(*mods)

    def forward(self, x):
        out = self.conv1(x)
        if self.bn1 is not None:
            out = F.relu(self.bn1(out))
        for i in range(1, 5):
            out = getattr(self, f"layer{i}")(out)
        return self.linear(F.adaptive_avg_pool2d(out, 1).flatten(1))


def PreActResNet18(num_classes=10):
    return PreActResNet(PreActBlock, [2, 2, 2, 2], num_classes)


# ------------------------------------------------------------------ SENet18

class SEBlock(PreActBlock):
    def __init__(self, cin, planes, stride=1):
        super().__init__(cin, planes, stride)
        self.fc1 = nn.Conv2d(planes, planes // 16, 1)
        self.fc2 = nn.Conv2d(planes // 16, planes, 1)

    def forward(self, x):
        out = F.relu(self.bn1(x))
        sc = self.shortcut(out) if self.shortcut is not None else x
        out = self.conv2(F.relu(self.bn2(self.conv1(out))))
        w = torch.sigmoid(self.fc2(F.relu(self.fc1(F.adaptive_avg_pool2d(out, 1)))))
        return out * w + sc


def SENet18(num_classes=10):
    """Pre-activation SE blocks behind a conv + BatchNorm stem (reference ``models/senet.py``)."""
    return PreActResNet(SEBlock, [2, 2, 2, 2], num_classes, stem_bn=True)


# ------------------------------------------------------------------ GoogLeNet

def conv_b_bn(cin, cout, k):
    """conv (with bias, as the reference GoogLeNet) + BatchNorm + ReLU, flattened into the caller."""
    return [nn.Conv2d(cin, cout, k, 1, (k - 1) // 2), nn.BatchNorm2d(cout), nn.ReLU(True)]


class Inception(nn.Module):
    def __init__(self, cin, n1, n3r, n3, n5r, n5, pool):
        super().__init__()
        self.b1 = nn.Sequential(*conv_b_bn(cin, n1, 1))
        self.b2 = nn.Sequential(*conv_b_bn(cin, n3r, 1), *conv_b_bn(n3r, n3, 3))
        self.b3 = nn.Sequential(*conv_b_bn(cin, n5r, 1), *conv_b_bn(n5r, n5, 3), *conv_b_bn(n5, n5, 3))
        self.b4 = nn.Sequential(nn.MaxPool2d(3, 1, 1), *conv_b_bn(cin, pool, 1))

    def forward(self, x):
        return torch.cat([self.b1(x), self.b2(x), self.b3(x), self.b4(x)], 1)


class GoogLeNet(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.pre = nn.Sequential(*conv_b_bn(3, 192, 3))
        cfg = [(192, 64, 96, 128, 16, 32, 32), (256, 128, 128, 192, 32, 96, 64), "M",
               (480, 192, 96, 208, 16, 48, 64), (512, 160, 112, 224, 24, 64, 64), (512, 128, 128, 256, 24, 64, 64),
               (512, 112, 144, 288, 32, 64, 64), (528, 256, 160, 320, 32, 128, 128), "M",
               (832, 256, 160, 320, 32, 128, 128), (832, 384, 192, 384, 48, 128, 128)]
        self.body = nn.Sequential(*[nn.MaxPool2d(3, 2, 1) if c == "M" else Inception(*c) for c in cfg])
        self.linear = nn.Linear(1024, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.body(self.pre(x)), 1).flatten(1))


# ------------------------------------------------------------------ DenseNet

class DenseLayer(nn.Module):
    def __init__(self, cin, growth):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(cin)
        self.conv1 = nn.Conv2d(cin, 4 * growth, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(4 * growth)
        self.conv2 = nn.Conv2d(4 * growth, growth, 3, 1, 1, bias=False)

    def forward(self, x):
        out = self.conv2(F.relu(self.bn2(self.conv1(F.relu(self.bn1(x))))))
        return torch.cat([out, x], 1)


class DenseNet(nn.Module):
    def __init__(self, blocks, growth=32, reduction=0.5, num_classes=10):
        super().__init__()
        c = 2 * growth
        self.conv1 = nn.Conv2d(3, c, 3, 1, 1, bias=False)
        stages = []
        for i, n in enumerate(blocks):
            layers = []
            for _ in range(n):
                layers.append(DenseLayer(c, growth))
                c += growth
            stages.append(nn.Sequential(*layers))
            if i < len(blocks) - 1:
                out = int(math.floor(c * reduction))
                stages.append(nn.Sequential(nn.BatchNorm2d(c), nn.ReLU(inplace=True),
                                            nn.Conv2d(c, out, 1, bias=False), nn.AvgPool2d(2)))
                c = out
        self.features = nn.Sequential(*stages)
        self.bn = nn.BatchNorm2d(c)
        self.linear = nn.Linear(c, num_classes)

    def forward(self, x):
        out = F.relu(self.bn(self.features(self.conv1(x))))
        return self.linear(F.adaptive_avg_pool2d(out, 1).flatten(1))


def DenseNet121(num_classes=10):
    return DenseNet([6, 12, 24, 16], 32, num_classes=num_classes)


# ------------------------------------------------------------------ ResNeXt29

class ResNeXtBlock(nn.Module):
    def __init__(self, cin, cardinality, width, stride):
        super().__init__()
        gw = cardinality * width
        self.body = nn.Sequential(conv_bn(cin, gw, 1), conv_bn(gw, gw, 3, stride, groups=cardinality),
                                  conv_bn(gw, 2 * gw, 1, act=False))
        self.shortcut = None
        if stride != 1 or cin != 2 * gw:
            self.shortcut = conv_bn(cin, 2 * gw, 1, stride, act=False)

    def forward(self, x):
        sc = x if self.shortcut is None else self.shortcut(x)
        return F.relu(self.body(x) + sc)


class ResNeXt29(nn.Module):
    def __init__(self, cardinality, width, num_classes=10):
        super().__init__()
        self.stem = conv_bn(3, 64, 1)
        cin, stages = 64, []
        for stride in (1, 2, 2):
            blocks = []
            for s in (stride, 1, 1):
                blocks.append(ResNeXtBlock(cin, cardinality, width, s))
                cin = 2 * cardinality * width
            stages.append(nn.Sequential(*blocks))
            width *= 2
        self.stages = nn.Sequential(*stages)
        self.linear = nn.Linear(cin, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.stages(self.stem(x)), 1).flatten(1))


def ResNeXt29_2x64d(num_classes=10):
    return ResNeXt29(2, 64, num_classes)


def ResNeXt29_4x64d(num_classes=10):
    return ResNeXt29(4, 64, num_classes)


def ResNeXt29_32x4d(num_classes=10):
    return ResNeXt29(32, 4, num_classes)


# ------------------------------------------------------------------ MobileNet v1 / v2

class MobileNet(nn.Module):
    CFG = [64, (128, 2), 128, (256, 2), 256, (512, 2), 512, 512, 512, 512, 512, (1024, 2), 1024]

    def __init__(self, num_classes=10):
        super().__init__()
        layers, cin = [conv_bn(3, 32, 3)], 32
        for c in self.CFG:
            out, s = (c, 1) if isinstance(c, int) else c
            layers += [conv_bn(cin, cin, 3, s, groups=cin), conv_bn(cin, out, 1)]
            cin = out
        self.features = nn.Sequential(*layers)
        self.linear = nn.Linear(1024, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.features(x), 1).flatten(1))


class InvertedResidual(nn.Module):
    def __init__(self, cin, cout, expansion, stride):
        super().__init__()
        hid = cin * expansion
        self.use_res = stride == 1 and cin == cout
        self.body = nn.Sequential(conv_bn(cin, hid, 1), conv_bn(hid, hid, 3, stride, groups=hid),
                                  conv_bn(hid, cout, 1, act=False))
        self.proj = None
        if stride == 1 and cin != cout:
            self.proj = conv_bn(cin, cout, 1, act=False)

    def forward(self, x):
        out = self.body(x)
        if self.use_res:
            return out + x
        if self.proj is not None:
            return out + self.proj(x)
        return out


class MobileNetV2(nn.Module):
    CFG = [(1, 16, 1, 1), (6, 24, 2, 1), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]

    def __init__(self, num_classes=10):
        super().__init__()
        layers, cin = [conv_bn(3, 32, 3)], 32
        for t, c, n, s in self.CFG:
            for i in range(n):
                layers.append(InvertedResidual(cin, c, t, s if i == 0 else 1))
                cin = c
        layers.append(conv_bn(cin, 1280, 1))
        self.features = nn.Sequential(*layers)
        self.linear = nn.Linear(1280, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.features(x), 1).flatten(1))


# ------------------------------------------------------------------ DPN

class DPNBottleneck(nn.Module):
    def __init__(self, cin, mid, out, dense, stride, first):
        super().__init__()
        self.out, self.dense = out, dense
        self.body = nn.Sequential(conv_bn(cin, mid, 1), conv_bn(mid, mid, 3, stride, groups=32),
                                  conv_bn(mid, out + dense, 1, act=False))
        self.shortcut = conv_bn(cin, out + dense, 1, stride, act=False) if first else None

    def forward(self, x):
        y = self.body(x)
        sc = x if self.shortcut is None else self.shortcut(x)
        d = self.out
        return F.relu(torch.cat([sc[:, :d] + y[:, :d], sc[:, d:], y[:, d:]], 1))


class DPN(nn.Module):
    def __init__(self, mids, outs, blocks, dense, num_classes=10):
        super().__init__()
        self.stem = conv_bn(3, 64, 3)
        cin, stages = 64, []
        for i, (m, o, n, dd) in enumerate(zip(mids, outs, blocks, dense)):
            layers = []
            for j in range(n):
                stride = (1 if i == 0 else 2) if j == 0 else 1
                layers.append(DPNBottleneck(cin, m, o, dd, stride, j == 0))
                cin = o + (j + 2) * dd
            stages.append(nn.Sequential(*layers))
        self.stages = nn.Sequential(*stages)
        self.linear = nn.Linear(cin, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.stages(self.stem(x)), 1).flatten(1))


def DPN26(num_classes=10):
    return DPN((96, 192, 384, 768), (256, 512, 1024, 2048), (2, 2, 2, 2), (16, 32, 24, 128), num_classes)


def DPN92(num_classes=10):
    return DPN((96, 192, 384, 768), (256, 512, 1024, 2048), (3, 4, 20, 3), (16, 32, 24, 128), num_classes)


# ------------------------------------------------------------------ ShuffleNet v1 / v2

def channel_shuffle(x, groups):
    b, c, h, w = x.shape
    return x.view(b, groups, c // groups, h, w).transpose(1, 2).reshape(b, c, h, w)


class ShuffleUnit(nn.Module):
    def __init__(self, cin, cout, stride, groups):
        super().__init__()
        self.stride, self.groups = stride, groups
        mid = cout // 4
        g = 1 if cin == 24 else groups
        self.conv1 = conv_bn(cin, mid, 1, groups=g)
        self.conv2 = conv_bn(mid, mid, 3, stride, groups=mid, act=False)
        self.conv3 = conv_bn(mid, cout - (cin if stride == 2 else 0), 1, groups=groups, act=False)

    def forward(self, x):
        out = self.conv3(self.conv2(channel_shuffle(self.conv1(x), self.groups)))
        if self.stride == 2:
            return F.relu(torch.cat([out, F.avg_pool2d(x, 3, 2, 1)], 1))
        return F.relu(out + x)


class ShuffleNet(nn.Module):
    def __init__(self, outs, blocks, groups, num_classes=10):
        super().__init__()
        self.stem = conv_bn(3, 24, 1)
        cin, layers = 24, []
        for o, n in zip(outs, blocks):
            for j in range(n):
                layers.append(ShuffleUnit(cin, o, 2 if j == 0 else 1, groups))
                cin = o
        self.body = nn.Sequential(*layers)
        self.linear = nn.Linear(cin, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.body(self.stem(x)), 1).flatten(1))


def ShuffleNetG2(num_classes=10):
    return ShuffleNet((200, 400, 800), (4, 8, 4), 2, num_classes)


def ShuffleNetG3(num_classes=10):
    return ShuffleNet((240, 480, 960), (4, 8, 4), 3, num_classes)


class ShuffleV2Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.stride = stride
        half = cout // 2
        if stride == 1:
            self.branch = nn.Sequential(conv_bn(half, half, 1), conv_bn(half, half, 3, groups=half, act=False),
                                        conv_bn(half, half, 1))
            self.left = None
        else:
            self.left = nn.Sequential(conv_bn(cin, cin, 3, 2, groups=cin, act=False), conv_bn(cin, half, 1))
            self.branch = nn.Sequential(conv_bn(cin, half, 1), conv_bn(half, half, 3, 2, groups=half, act=False),
                                        conv_bn(half, half, 1))

    def forward(self, x):
        if self.stride == 1:
            a, b = x.chunk(2, 1)
            out = torch.cat([a, self.branch(b)], 1)
        else:
            out = torch.cat([self.left(x), self.branch(x)], 1)
        return channel_shuffle(out, 2)


class ShuffleNetV2(nn.Module):
    SIZES = {0.5: (48, 96, 192, 1024), 1: (116, 232, 464, 1024), 1.5: (176, 352, 704, 1024),
             2: (224, 488, 976, 2048)}

    def __init__(self, net_size=1, num_classes=10):
        super().__init__()
        outs = self.SIZES[net_size]
        self.stem = conv_bn(3, 24, 3)
        cin, layers = 24, []
        for o, n in zip(outs[:3], (3, 7, 3)):
            layers.append(ShuffleV2Block(cin, o, 2))
            layers += [ShuffleV2Block(o, o, 1) for _ in range(n)]
            cin = o
        layers.append(conv_bn(cin, outs[3], 1))
        self.body = nn.Sequential(*layers)
        self.linear = nn.Linear(outs[3], num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.body(self.stem(x)), 1).flatten(1))


# ------------------------------------------------------------------ EfficientNet-B0

class MBConv(nn.Module):
    """Expansion 1x1 -> depthwise kxk -> squeeze-excitation (swish) -> projection 1x1.

    Parameter list as the reference ``models/efficientnet.py`` Block: the expansion
    conv + BatchNorm exist even when expansion == 1 (unused in the forward), and the
    SE width is a quarter of the block INPUT channels. The reference computes the
    drop-connect rate from a block counter it never increments (every rate is 0);
    ``drop`` keeps that default."""

    def __init__(self, cin, cout, expansion, k, stride, se_ratio=0.25, drop=0.0):
        super().__init__()
        hid = cin * expansion
        self.expansion = expansion
        self.skip = stride == 1 and cin == cout
        self.conv1 = nn.Conv2d(cin, hid, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(hid)
        self.conv2 = nn.Conv2d(hid, hid, k, stride, k // 2, groups=hid, bias=False)
        self.bn2 = nn.BatchNorm2d(hid)
        se = int(cin * se_ratio)
        self.se1, self.se2 = nn.Conv2d(hid, se, 1), nn.Conv2d(se, hid, 1)
        self.conv3 = nn.Conv2d(hid, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.drop = drop

    def forward(self, x):
        out = x if self.expansion == 1 else F.silu(self.bn1(self.conv1(x)))
        out = F.silu(self.bn2(self.conv2(out)))
        out = out * torch.sigmoid(self.se2(F.silu(self.se1(F.adaptive_avg_pool2d(out, 1)))))
        out = self.bn3(self.conv3(out))
        if self.skip:
            if self.training and self.drop > 0:
                keep = torch.rand(x.shape[0], 1, 1, 1, device=x.device) >= self.drop
                out = out * keep / (1 - self.drop)
            out = out + x
        return out


class EfficientNetB0(nn.Module):
    CFG = [(1, 16, 1, 3, 1), (6, 24, 2, 3, 2), (6, 40, 2, 5, 2), (6, 80, 3, 3, 2), (6, 112, 3, 5, 1),
           (6, 192, 4, 5, 2), (6, 320, 1, 3, 1)]

    def __init__(self, num_classes=10, drop_connect=0.0):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        cin, layers = 32, []
        total = sum(c[2] for c in self.CFG)
        b = 0
        for t, c, n, k, s in self.CFG:
            for i in range(n):
                layers.append(MBConv(cin, c, t, k, s if i == 0 else 1, drop=drop_connect * b / total))
                cin, b = c, b + 1
        self.layers = nn.Sequential(*layers)
        self.linear = nn.Linear(cin, num_classes)

    def forward(self, x):
        out = self.layers(F.silu(self.bn1(self.conv1(x))))
        return self.linear(F.dropout(F.adaptive_avg_pool2d(out, 1).flatten(1), 0.2, self.training))


# ------------------------------------------------------------------ RegNetX

class RegNetXBlock(nn.Module):
    def __init__(self, cin, cout, stride, group_width, bottleneck=1):
        super().__init__()
        w = cout // bottleneck
        self.body = nn.Sequential(conv_bn(cin, w, 1), conv_bn(w, w, 3, stride, groups=w // group_width),
                                  conv_bn(w, cout, 1, act=False))
        self.shortcut = None
        if stride != 1 or cin != cout:
            self.shortcut = conv_bn(cin, cout, 1, stride, act=False)

    def forward(self, x):
        sc = x if self.shortcut is None else self.shortcut(x)
        return F.relu(self.body(x) + sc)


class RegNetX(nn.Module):
    def __init__(self, depths, widths, strides, group_width, num_classes=10):
        super().__init__()
        self.stem = conv_bn(3, 64, 3)
        cin, layers = 64, []
        for d, w, s in zip(depths, widths, strides):
            for i in range(d):
                layers.append(RegNetXBlock(cin, w, s if i == 0 else 1, group_width))
                cin = w
        self.body = nn.Sequential(*layers)
        self.linear = nn.Linear(cin, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.body(self.stem(x)), 1).flatten(1))


def RegNetX_200MF(num_classes=10):
    return RegNetX((1, 1, 4, 7), (24, 56, 152, 368), (1, 1, 2, 2), 8, num_classes)


def RegNetX_400MF(num_classes=10):
    return RegNetX((1, 2, 7, 12), (32, 64, 160, 384), (1, 1, 2, 2), 16, num_classes)


# ------------------------------------------------------------------ PNASNet

class SepConv(nn.Module):
    def __init__(self, cin, cout, k, stride):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=cin, bias=False)
        self.bn = nn.BatchNorm2d(cout)

    def forward(self, x):
        return self.bn(self.conv(x))


class PNASCellA(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.stride = stride
        self.sep = SepConv(cin, cout, 7, stride)
        self.reduce = conv_bn(cin, cout, 1, act=False) if stride == 2 else None

    def forward(self, x):
        y1 = self.sep(x)
        y2 = F.max_pool2d(x, 3, self.stride, 1)
        if self.reduce is not None:
            y2 = self.reduce(y2)
        return F.relu(y1 + y2)


class PNASCellB(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.stride = stride
        self.sep1, self.sep2, self.sep3 = SepConv(cin, cout, 7, stride), SepConv(cin, cout, 3, stride), \
            SepConv(cin, cout, 5, stride)
        self.reduce = conv_bn(cin, cout, 1, act=False) if stride == 2 else None
        self.mix = conv_bn(2 * cout, cout, 1)

    def forward(self, x):
        y1, y2 = self.sep1(x), self.sep2(x)
        y3 = F.max_pool2d(x, 3, self.stride, 1)
        if self.reduce is not None:
            y3 = self.reduce(y3)
        y4 = self.sep3(x)
        return self.mix(torch.cat([F.relu(y1 + y2), F.relu(y3 + y4)], 1))


class PNASNet(nn.Module):
    def __init__(self, cell, planes, cells_per_stage=6, num_classes=10):
        super().__init__()
        self.stem = conv_bn(3, planes, 3)
        cin, layers = planes, []
        for stage in range(3):
            if stage > 0:
                layers.append(cell(cin, cin * 2, 2))
                cin *= 2
            layers += [cell(cin, cin, 1) for _ in range(cells_per_stage)]
        self.body = nn.Sequential(*layers)
        self.linear = nn.Linear(cin, num_classes)

    def forward(self, x):
        return self.linear(F.adaptive_avg_pool2d(self.body(self.stem(x)), 1).flatten(1))


def PNASNetA(num_classes=10):
    return PNASNet(PNASCellA, 44, num_classes=num_classes)


def PNASNetB(num_classes=10):
    return PNASNet(PNASCellB, 32, num_classes=num_classes)


# ------------------------------------------------------------------ VGG

VGG_CFG = {"VGG11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
           "VGG13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
           "VGG16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
           "VGG19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
                     512, 512, 512, 512, "M"]}


def _vgg_features(cfg, bn=True):
    layers, cin = [], 3
    for c in cfg:
        if c == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers += [nn.Conv2d(cin, c, 3, padding=1)] + ([nn.BatchNorm2d(c)] if bn else []) + [nn.ReLU(inplace=True)]
            cin = c
    return nn.Sequential(*layers)


class VGG(nn.Module):
    """CIFAR VGG (BN, one linear layer) — reference ``models/vgg.py``."""

    def __init__(self, vgg_name="VGG16", num_classes=10):
        super().__init__()
        self.features = _vgg_features(VGG_CFG[vgg_name])
        self.classifier = nn.Linear(512, num_classes)

    def forward(self, x):
        return self.classifier(self.features(x).flatten(1))


class ImageNetVGG(nn.Module):
    """torchvision VGG16/19 architecture (no BN, 4096-wide classifier), as the
    reference instantiates for ``vgg16`` / ``vgg19``."""

    def __init__(self, vgg_name="VGG16", num_classes=1000):
        super().__init__()
        self.features = _vgg_features(VGG_CFG[vgg_name], bn=False)
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(nn.Linear(512 * 49, 4096), nn.ReLU(True), nn.Dropout(),
                                        nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(),
                                        nn.Linear(4096, num_classes))

    def forward(self, x):
        return self.classifier(self.avgpool(self.features(x)).flatten(1))
