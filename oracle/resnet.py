"""ResNet-50 v1.5 restated in plain torch.nn — TEST INFRASTRUCTURE (oracle), never product code.

The reference builds its backbone with ``torchvision.models.resnet50(weights="DEFAULT")``
(``argus/models.py:43``). torchvision is an unpinned third-party dependency
(``pyproject.toml:27`` ``torchvision>=0.15.2``) that is not present in ``/root/reference`` nor in this
image, so its published ResNet-50 definition is restated here:

- Bottleneck with the stride on the 3x3 conv (v1.5), expansion 4, ``bias=False`` convs;
- stem 7x7/2 p3 conv -> BN -> ReLU -> 3x3/2 p1 max-pool; stages (3, 4, 6, 3);
- the 1x1 downsample ``Sequential(conv, BN)`` is constructed *before* the first block of a stage
  (matters for RNG consumption order), but registered after ``bn3``/``relu`` of that block;
- init: every Conv2d first gets its default ``reset_parameters`` (kaiming_uniform a=sqrt 5) at
  construction, then ``kaiming_normal_(mode="fan_out", nonlinearity="relu")`` in ``modules()`` order;
  BN weight 1, bias 0; Linear default init. ``zero_init_residual=False``.

Pretrained weights (``weights="DEFAULT"``) are a network download and are unavailable offline:
seeded random init is used instead (documented in DESIGN.md).
"""
from __future__ import annotations

import torch
import torch.nn as nn


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out = out + identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(
                conv1x1(self.inplanes, planes * Bottleneck.expansion, stride),
                nn.BatchNorm2d(planes * Bottleneck.expansion),
            )
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = self.avgpool(x)
        x = torch.flatten(x, 1)
        return self.fc(x)


def resnet50(weights=None, **kwargs) -> ResNet:
    """Signature-compatible stand-in for ``torchvision.models.resnet50``; ``weights`` is ignored."""
    return ResNet((3, 4, 6, 3), **kwargs)
