from garfield_amd.models import *  # noqa: F401,F403
from garfield_amd.models.nets import CNNet, Cifarnet, LeNet, Net, PimaNet  # noqa: F401
from garfield_amd.models.resnet import ResNet18, ResNet34, ResNet50, ResNet101, ResNet152  # noqa: F401
