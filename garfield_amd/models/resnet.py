"""ResNet families.

* ``cifar_resnet*``: CIFAR-style ResNets with a 3x3 stem (the reference's local
  ``models/resnet.py:73-124``, used for ``resnet18``).
* ``imagenet_resnet*``: the torchvision architecture (7x7 stride-2 stem + max
  pool, Bottleneck v1.5 with the stride on the 3x3 conv), which the reference
  instantiates for ``resnet34/50/152`` via ``torchvision.models`` (``garfieldpp/
  tools.py:66-88``). torchvision is not a dependency here; this is an
  architecture-identical implementation (``resnet50`` with 10 classes has
  23,528,522 parameters) with torchvision's initialisation.

Both take ``NCHW`` input; call ``.to(memory_format=torch.channels_last)`` on the
model and input to run MIOpen's NHWC kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)), inplace=True)
        out = self.bn2(self.conv2(out))
        sc = x if self.downsample is None else self.downsample(x)
        return F.relu(out + sc, inplace=True)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)), inplace=True)
        out = F.relu(self.bn2(self.conv2(out)), inplace=True)
        out = self.bn3(self.conv3(out))
        sc = x if self.downsample is None else self.downsample(x)
        return F.relu(out + sc, inplace=True)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=10, stem="imagenet", in_channels=3):
        super().__init__()
        self.in_planes = 64
        if stem == "imagenet":
            self.conv1 = nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
            self.maxpool = nn.MaxPool2d(3, 2, 1)
        else:
            self.conv1 = nn.Conv2d(in_channels, 64, 3, 1, 1, bias=False)
            self.maxpool = nn.Identity()
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make(block, 64, layers[0], 1)
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make(self, block, planes, blocks, stride):
        down = None
        if stride != 1 or self.in_planes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.in_planes, planes * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.in_planes, planes, stride, down)]
        self.in_planes = planes * block.expansion
        layers += [block(self.in_planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(F.relu(self.bn1(self.conv1(x)), inplace=True))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


_CFG = {18: (BasicBlock, [2, 2, 2, 2]), 34: (BasicBlock, [3, 4, 6, 3]), 50: (Bottleneck, [3, 4, 6, 3]),
        101: (Bottleneck, [3, 4, 23, 3]), 152: (Bottleneck, [3, 8, 36, 3]),
        200: (Bottleneck, [3, 24, 36, 3])}


def imagenet_resnet(depth: int, num_classes: int = 1000) -> ResNet:
    block, layers = _CFG[depth]
    return ResNet(block, layers, num_classes, stem="imagenet")


def cifar_resnet(depth: int, num_classes: int = 10) -> ResNet:
    block, layers = _CFG[depth]
    return ResNet(block, layers, num_classes, stem="cifar")


def ResNet18(num_classes=10):
    return cifar_resnet(18, num_classes)


def ResNet34(num_classes=10):
    return cifar_resnet(34, num_classes)


def ResNet50(num_classes=10):
    return cifar_resnet(50, num_classes)


def ResNet101(num_classes=10):
    return cifar_resnet(101, num_classes)


def ResNet152(num_classes=10):
    return cifar_resnet(152, num_classes)
