"""Model zoo with the reference's ``select_model`` names.

Reference: ``pytorch_impl/libs/garfieldpp/tools.py:59-105`` and ``models/*.py``.
``resnet18`` is the CIFAR-stem ResNet-18 (reference-local model); ``resnet34/50/152``,
``vgg16/19`` and ``inception`` follow the torchvision architectures the reference
instantiates (implemented here, torchvision is not required).
"""
from __future__ import annotations

import importlib

import torch.nn as nn

NUM_CLASSES = {"cifar10": 10, "cifar100": 100, "mnist": 10, "imagenet": 1000, "pima": 1, "synthetic": 10}

# name -> (module, attribute, kwargs)
_REGISTRY = {
    "convnet": ("nets", "Net", {}),
    "cifarnet": ("nets", "Cifarnet", {}),
    "cnn": ("nets", "CNNet", {}),
    "lenet": ("nets", "LeNet", {}),
    "pimanet": ("nets", "PimaNet", {}),
    "mlp": ("nets", "MLP", {}),
    "resnet18": ("resnet", "ResNet18", {}),
    "cifar_resnet34": ("resnet", "ResNet34", {}),
    "cifar_resnet50": ("resnet", "ResNet50", {}),
    "cifar_resnet101": ("resnet", "ResNet101", {}),
    "cifar_resnet152": ("resnet", "ResNet152", {}),
    "resnet34": ("resnet", "imagenet_resnet", {"depth": 34}),
    "resnet50": ("resnet", "imagenet_resnet", {"depth": 50}),
    "resnet101": ("resnet", "imagenet_resnet", {"depth": 101}),
    "resnet152": ("resnet", "imagenet_resnet", {"depth": 152}),
    "resnet200": ("resnet", "imagenet_resnet", {"depth": 200}),
    "inception_v3": ("inception", "InceptionV3", {}),
    "inception": ("inception", "InceptionV3", {}),
    "preactresnet18": ("zoo", "PreActResNet18", {}),
    "googlenet": ("zoo", "GoogLeNet", {}),
    "densenet121": ("zoo", "DenseNet121", {}),
    "resnext29": ("zoo", "ResNeXt29_2x64d", {}),
    "resnext29_4x64d": ("zoo", "ResNeXt29_4x64d", {}),
    "resnext29_32x4d": ("zoo", "ResNeXt29_32x4d", {}),
    "mobilenet": ("zoo", "MobileNet", {}),
    "mobilenetv2": ("zoo", "MobileNetV2", {}),
    "dpn26": ("zoo", "DPN26", {}),
    "dpn92": ("zoo", "DPN92", {}),
    "shufflenetg2": ("zoo", "ShuffleNetG2", {}),
    "shufflenetg3": ("zoo", "ShuffleNetG3", {}),
    "shufflenetv2": ("zoo", "ShuffleNetV2", {}),
    "senet18": ("zoo", "SENet18", {}),
    "efficientnetb0": ("zoo", "EfficientNetB0", {}),
    "regnetx200": ("zoo", "RegNetX_200MF", {}),
    "regnetx400": ("zoo", "RegNetX_400MF", {}),
    "pnasneta": ("zoo", "PNASNetA", {}),
    "pnasnetb": ("zoo", "PNASNetB", {}),
    "vgg11_cifar": ("zoo", "VGG", {"vgg_name": "VGG11"}),
    "vgg16_cifar": ("zoo", "VGG", {"vgg_name": "VGG16"}),
    "vgg19_cifar": ("zoo", "VGG", {"vgg_name": "VGG19"}),
    "vgg16": ("zoo", "ImageNetVGG", {"vgg_name": "VGG16"}),
    "vgg19": ("zoo", "ImageNetVGG", {"vgg_name": "VGG19"}),
}


def register_model(name: str, module: str, attr: str, **kwargs) -> None:
    _REGISTRY[name] = (module, attr, kwargs)


def available_models() -> list[str]:
    return sorted(_REGISTRY)


def build_model(name: str, num_classes: int | None = None, dataset: str | None = None) -> nn.Module:
    """Instantiate model ``name`` with ``num_classes`` (or the dataset's class count)."""
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name!r}; available: {available_models()}")
    if num_classes is None:
        num_classes = NUM_CLASSES.get(dataset or "cifar10", 10)
    mod, attr, kw = _REGISTRY[name]
    fn = getattr(importlib.import_module(f"garfield_amd.models.{mod}"), attr)
    return fn(num_classes=num_classes, **kw)


def num_parameters(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
