"""ResNet-18/34/50/101/152 with torchvision parameter naming.

The reference builds ``torchvision.models.resnet18(pretrained=False)``
(``resnet/main.py:76``); torchvision is not a dependency here, so the
architecture is re-specified: stem conv7x7/s2 + BN + ReLU +
maxpool3x3/s2, four stages of BasicBlock/Bottleneck (v1.5: stride on the 3x3),
global average pool, fc.  Parameter names, shapes, init and therefore the
``state_dict`` layout are identical to torchvision's, so a
checkpoint written here loads into a torchvision model and vice versa.

Two execution back-ends share the same ``nn.Parameter``s:

* ``impl="torch"``  -- plain ATen ops (NCHW or channels_last, autocast).  This is
  the stock path the reference runs and the numerics oracle for tests.
* ``impl="native"`` -- the MI355X path: activations are NHWC bf16, every
  conv is a fused ``conv -> BN(batch stats) -> (+residual) -> ReLU`` unit backed by
  the hand-written HIP kernels in ``csrc/kernels`` (see ``ops/``).  Conv weights
  are kept in ``channels_last`` memory (= KRSC, the implicit-GEMM B layout) so the
  kernels read the fp32 master weights and write weight gradients without any
  layout shuffles.
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn

from .. import ops

__all__ = [
    "ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet34", "resnet50",
    "resnet101", "resnet152", "build_model", "MODEL_SPECS",
]


def _conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def _conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)

    def forward_native(self, x: torch.Tensor, tail: bool = False) -> torch.Tensor:
        if x.is_cuda:  # one fused autograd node per block on the device path
            m = self._modules  # direct dict reads: nn.Module.__getattr__ is a slow fallback path
            d = m.get("downsample")  # None is a plain attribute, not in _modules
            ds = (d[0], d[1]) if d is not None else None
            return ops.residual_block(x, [(m["conv1"], m["bn1"]), (m["conv2"], m["bn2"])], ds, tail)
        out = ops.conv_bn(x, self.conv1, self.bn1, relu=True)
        identity = x
        if self.downsample is not None:
            identity = ops.conv_bn(x, self.downsample[0], self.downsample[1], relu=False)
        return ops.conv_bn(out, self.conv2, self.bn2, relu=True, residual=identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = _conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv1x1(width, planes * self.expansion)
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
        return self.relu(out + identity)

    def forward_native(self, x: torch.Tensor, tail: bool = False) -> torch.Tensor:
        if x.is_cuda:  # one fused autograd node per block on the device path
            m = self._modules  # direct dict reads: nn.Module.__getattr__ is a slow fallback path
            d = m.get("downsample")  # None is a plain attribute, not in _modules
            ds = (d[0], d[1]) if d is not None else None
            return ops.residual_block(
                x, [(m["conv1"], m["bn1"]), (m["conv2"], m["bn2"]), (m["conv3"], m["bn3"])], ds, tail)
        identity = x
        if self.downsample is not None:
            identity = ops.conv_bn(x, self.downsample[0], self.downsample[1], relu=False)
        out = ops.conv_bn(x, self.conv1, self.bn1, relu=True)
        out = ops.conv_bn(out, self.conv2, self.bn2, relu=True)
        return ops.conv_bn(out, self.conv3, self.bn3, relu=True, residual=identity)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int],
                 num_classes: int = 1000, impl: str = "torch"):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)

        # torchvision init: kaiming_normal(fan_out, relu) for convs, BN gamma=1 beta=0,
        # nn.Linear keeps its default init.  zero_init_residual=False.
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self.impl = "torch"
        self.set_impl(impl)

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                _conv1x1(self.inplanes, planes * block.expansion, stride),
                nn.BatchNorm2d(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    # ------------------------------------------------------------------ impl
    def set_impl(self, impl: str) -> "ResNet":
        """Switch execution back-end.  ``native`` stores conv weights channels_last
        (KRSC memory order) -- a pure memory-format change, values/shapes unchanged."""
        if impl not in ("torch", "native"):
            raise ValueError(f"unknown impl {impl!r}")
        self.impl = impl
        ops.forget_bn_modules(self)  # re-collected at the next device forward
        if impl == "native":
            for m in self.modules():
                if isinstance(m, nn.Conv2d):
                    with torch.no_grad():
                        m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
        return self

    # --------------------------------------------------------------- forward
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.impl == "native":
            return self.forward_native(x)
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)

    def forward_native(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:  # every BN counter bumped by one launch (see ops.bump_bn_counters)
            with ops.bump_bn_counters(self):
                return self._forward_native(x)
        return self._forward_native(x)

    def _forward_native(self, x: torch.Tensor) -> torch.Tensor:
        # NCHW fp32 image (or an NHWC bf16 tensor already prepared by the data
        # pipeline) -> NHWC bf16 with C padded to the kernels' 8-channel granule.
        if x.is_cuda:  # bf16 conv-weight mirror of the DDP flat space (refreshed if stale)
            sp = getattr(self.conv1.weight, "_pdt_flat", None)
            mirror = sp.mirror() if sp is not None else None
            if mirror is not None:
                mirror.ensure()
        if x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and x.is_floating_point():
            # super-pixel stem conv, then BN + ReLU + max pool in one pass (fused.py)
            x = ops.stem_conv_bn_pool(x, self.conv1, self.bn1, self.maxpool)
        else:
            if x.dim() == 4 and x.shape[1] == 3:
                x = ops.image_to_nhwc(x)
            x = ops.conv_bn(x, self.conv1, self.bn1, relu=True)
            x = ops.maxpool3x3s2(x)
        x = ops.fp8_attach(x, self.maxpool)  # e4m3 copy for fp8 convs (no-op unless ops.set_fp8)
        last = self.layer4[len(self.layer4) - 1]
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                x = blk.forward_native(x, blk is last)  # the tail block hands no BN backward on
        return ops.avgpool_linear(x, self.fc.weight, self.fc.bias)


MODEL_SPECS = {
    "resnet18": (BasicBlock, [2, 2, 2, 2]),
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
    "resnet101": (Bottleneck, [3, 4, 23, 3]),
    "resnet152": (Bottleneck, [3, 8, 36, 3]),
}


def build_model(arch: str = "resnet18", num_classes: int = 1000, impl: str = "torch") -> ResNet:
    if arch not in MODEL_SPECS:
        raise ValueError(f"unknown arch {arch!r}; choose from {sorted(MODEL_SPECS)}")
    block, layers = MODEL_SPECS[arch]
    return ResNet(block, layers, num_classes=num_classes, impl=impl)


def resnet18(**kw) -> ResNet:
    return build_model("resnet18", **kw)


def resnet34(**kw) -> ResNet:
    return build_model("resnet34", **kw)


def resnet50(**kw) -> ResNet:
    return build_model("resnet50", **kw)


def resnet101(**kw) -> ResNet:
    return build_model("resnet101", **kw)


def resnet152(**kw) -> ResNet:
    return build_model("resnet152", **kw)
