"""ResNet-50 (Bottleneck, [3, 4, 6, 3]) with torchvision-compatible module names.

Reference: ``torchvision.models.resnet50(num_classes=1000)`` NB03:560-570 and the
``ResNet(Bottleneck, [3,4,6,3])`` base of ``ModelParallelResNet50`` NB03:807-833
(SURVEY R20, K15). torchvision is not a dependency here, so the architecture is
defined directly; parameter count (25,557,032) and state_dict keys match
torchvision's so checkpoints interchange.

Execution on MI355X: convolutions and pooling run on MIOpen through PyTorch-ROCm
(the reference's cuDNN role; a hand-written conv stack is out of scope for this
harness and documented as such in SURVEY K15). Every BatchNorm is
``ops.norm.BatchNorm2d`` with its ReLU and the Bottleneck's residual add fused
(native NHWC kernels, csrc/kernels/batchnorm.hip, for channels_last
activations), and the classifier ``fc`` runs on the native MFMA Linear kernel.
``model.to(memory_format=torch.channels_last)`` keeps activations NHWC, the
layout MIOpen's fastest gfx950 conv solvers and the BN kernels use.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.conv import Conv2d
from ..ops.convbn import conv_bn_act
from ..ops.linear import Linear
from ..ops.norm import BatchNorm2d, MaxPool2d, bn_relu_maxpool, grad_link


def bn_act(bn: nn.Module, x: torch.Tensor, residual: torch.Tensor | None = None, relu: bool = False,
           link: bool = False):
    """``ReLU?(bn(x) + residual)``: fused for ops.norm.BatchNorm2d, composed for any other norm layer.
    ``link``: the residual is an identity shortcut from another fused BN (ops.norm.ResidualLink)."""
    if isinstance(bn, BatchNorm2d):
        return bn(x, residual, relu, link)
    y = bn(x)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    return Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation, groups=groups,
                     bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    return Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or BatchNorm2d
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def _down(self, x):
        ds = self.downsample
        if isinstance(ds, nn.Sequential) and len(ds) == 2 and isinstance(ds[0], nn.Conv2d):
            return conv_bn_act(ds[0], ds[1], x)  # stride 1 (layer1): BN statistics in the conv epilogue
        return ds(x)

    def forward(self, x):
        # downsample block: x feeds conv1 and the downsample conv; the downsample branch's input
        # gradient is summed inside the producing BN's backward (ops.norm.grad_link), not by autograd
        identity = x if self.downsample is None else self._down(grad_link(x))
        # 1x1 convs: the BN statistics come from the GEMM epilogue (ops.convbn) where it applies
        out = conv_bn_act(self.conv1, self.bn1, x, relu=True)
        out = bn_act(self.bn2, self.conv2(out), relu=True)
        # identity shortcut: the residual gradient goes straight into the producing BN's backward
        return conv_bn_act(self.conv3, self.bn3, out, residual=identity, relu=True, link=self.downsample is None)


class ResNet(nn.Module):
    def __init__(self, block=Bottleneck, layers=(3, 4, 6, 3), num_classes: int = 1000, zero_init_residual=False,
                 groups=1, width_per_group=64, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or BatchNorm2d
        self._norm_layer = norm_layer
        self.inplanes = 64
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        self.conv1 = Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, self.dilation,
                        norm_layer)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                dilation=self.dilation, norm_layer=norm_layer))
        return nn.Sequential(*layers)

    def _forward_impl(self, x):
        # stem: the BN apply + ReLU run inside the pool's loads (ops.norm.bn_relu_maxpool)
        x = bn_relu_maxpool(self.conv1(x), self.bn1, self.maxpool)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)

    def forward(self, x):
        return self._forward_impl(x)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, (3, 4, 6, 3), num_classes=num_classes, **kw)
