"""Parameter containers of the reference's resnet attribute encoder (network/resnet.py).

``MLAttrEncoderResnet()`` (resnet.py:147-149) builds ResNet(Bottleneck, [2, 2, 2, 2, 2, 2]) whose
submodule names give the ``encoder.*`` state_dict keys AEI_Net(backbone='resnet') loads.  The
modules here only hold parameters with those names and layouts; the computation runs inside the
native AEI_Net plan (aei_runtime.hip ``encoder_resnet``), so calling them directly raises.
"""
from __future__ import annotations

import math

import torch.nn as nn

PLANES = [32, 64, 128, 256, 512, 256]   # resnet.py:93-98


class Bottleneck(nn.Module):
    """1x1/s -> BN -> ReLU -> 3x3 -> BN -> ReLU -> 1x1 (x4) -> BN, + residual, ReLU (resnet.py:43-78)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        raise NotImplementedError("ghost_amd: the resnet encoder runs inside AEI_Net.forward / get_attr")


class ResNet(nn.Module):
    """Stem (conv0 7x7/s1, conv1 7x7/s2, BN + ReLU each) and six Bottleneck layers (resnet.py:81-120)."""

    def __init__(self, layers=(2, 2, 2, 2, 2, 2)):
        super().__init__()
        self.inplanes = 64
        self.conv0 = nn.Conv2d(3, 64, kernel_size=7, stride=1, padding=3, bias=False)
        self.bn0 = nn.BatchNorm2d(64)
        self.relu0 = nn.ReLU(inplace=True)
        self.conv1 = nn.Conv2d(64, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        for i, (planes, n) in enumerate(zip(PLANES, layers), 1):
            setattr(self, f"layer{i}", self._make_layer(planes, n, stride=2))
        for m in self.modules():   # the reference's init (resnet.py:100-106); overwritten by load_state_dict
            if isinstance(m, nn.Conv2d):
                fan = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2. / fan))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        self._owner = None

    def _make_layer(self, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, kernel_size=1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes * 4))
        mods = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        mods += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x):
        if self._owner is None:
            raise NotImplementedError("ghost_amd: call AEI_Net.get_attr (the encoder runs as part of the AEI_Net plan)")
        return self._owner().get_attr(x)


def MLAttrEncoderResnet(**kwargs):
    """resnet.py:147-149."""
    return ResNet((2, 2, 2, 2, 2, 2))
