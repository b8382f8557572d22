"""ResNet feature backbones -- drop-in for ``features/resnet_features.py``.

Same module tree / ``state_dict`` keys as the reference (``conv1``, ``bn1``,
``layer{1..4}.{j}.{conv,bn}{1,2,3}``, ``downsample.{0,1}``); layer3 and layer4 run at
stride 1 (``resnet_features.py:153-154``) so a 224x224 image gives a 28x28 grid.

Eval + no-grad forwards run on the HIP kernels (see ``resnet_hip.py``): BatchNorm folded
into the convolution weights at pack time, NHWC implicit-GEMM convolutions on MFMA with
bias / residual / ReLU fused into the epilogue.
"""
from __future__ import annotations

import warnings
from typing import Dict

import torch
import torch.nn as nn

from .backend import use_hip

Tensor = torch.Tensor


def conv3x3(in_planes: int, out_planes: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(in_planes: int, out_planes: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1
    num_layers = 2

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)

    def block_conv_info(self):
        return [3, 3], [self.stride, 1], [1, 1]


class Bottleneck(nn.Module):
    expansion = 4
    num_layers = 3

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)

    def block_conv_info(self):
        return [1, 3, 1], [1, self.stride, 1], [0, 1, 0]


class ResNet_features(nn.Module):
    """features/resnet_features.py:126-229 (avgpool / fc removed, layer3+4 stride 1)."""

    def __init__(self, block, layers, num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.kernel_sizes, self.strides, self.paddings = [7, 3], [2, 2], [3, 1]
        self.block = block
        self.layers = layers
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=1)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)
        self._hip_pack: Dict = {}
        # compute dtype of the HIP inference path: torch.float32 (exact, the reference's) or
        # torch.bfloat16 (BASELINE C3 build; features come back as bf16 NHWC-backed views)
        self.hip_dtype = torch.float32

    def _make_layer(self, block, planes, num_blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        blocks = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        blocks += [block(self.inplanes, planes) for _ in range(1, num_blocks)]
        for b in blocks:
            ks, ss, ps = b.block_conv_info()
            self.kernel_sizes += ks
            self.strides += ss
            self.paddings += ps
        return nn.Sequential(*blocks)

    def hip_steps(self, x):
        """The HIP forward as a block-by-block generator returning NHWC features."""
        from .resnet_hip import resnet_features_hip_steps
        return resnet_features_hip_steps(self, x, self._hip_pack)

    def forward(self, x):
        if use_hip(self):
            from .resnet_hip import resnet_features_hip
            from .convnext_features import nhwc_as_nchw
            return nhwc_as_nchw(resnet_features_hip(self, x, self._hip_pack))
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))

    def conv_info(self):
        return self.kernel_sizes, self.strides, self.paddings

    def num_layers(self):
        return self.block.num_layers * sum(self.layers) + 1

    def __repr__(self):
        return "resnet{}_features".format(self.num_layers() + 1)


def _make(block, layers, pretrained: bool, **kwargs):
    model = ResNet_features(block, layers, **kwargs)
    if pretrained:
        warnings.warn("ImageNet ResNet weights are unavailable offline (model_zoo download, "
                      "resnet_features.py:238-266); keeping random init -- load a checkpoint instead.")
    return model


def resnet18_features(pretrained=False, **kwargs):
    return _make(BasicBlock, [2, 2, 2, 2], pretrained, **kwargs)


def resnet34_features(pretrained=False, **kwargs):
    return _make(BasicBlock, [3, 4, 6, 3], pretrained, **kwargs)


def resnet50_features(pretrained=False, **kwargs):
    return _make(Bottleneck, [3, 4, 6, 3], pretrained, **kwargs)


def resnet50_features_inat(pretrained=False, **kwargs):
    return _make(Bottleneck, [3, 4, 6, 3], pretrained, **kwargs)


def resnet101_features(pretrained=False, **kwargs):
    return _make(Bottleneck, [3, 4, 23, 3], pretrained, **kwargs)


def resnet152_features(pretrained=False, **kwargs):
    return _make(Bottleneck, [3, 8, 36, 3], pretrained, **kwargs)
