"""ImageNet ResNets (ResNet-50/101/152) written for this framework.

The reference's ImageNet examples take these models from torchvision
(`examples/torch_imagenet_resnet.py:130-140` in the reference); torchvision is
not part of this image, so the architecture is built here.  It follows the
"v1.5" bottleneck (stride on the 3x3 convolution), which is what torchvision's
`resnet50()` builds, so the K-FAC layer inventory (53 Conv2d + 1 Linear for
ResNet-50, factor sizes in SURVEY.md section 2.3) is identical.

MI355X notes: the model is memory-format agnostic; `bench.py` runs it in
`channels_last` under bf16 autocast, which is the layout MIOpen's NHWC
kernels prefer on gfx950 (measured in profiles/).  Every BatchNorm, with the
ReLU and the residual add that follow it, runs through ops/bn.bn_act: fused
hand-written kernels (csrc/bn.hip) for bf16 channels_last training batches,
the stock modules otherwise (same parameters, buffers and state_dict).
"""
import torch
import torch.nn as nn

from ..ops.bn import bn_act

__all__ = ['ResNet', 'Bottleneck', 'BasicBlock', 'resnet_tiny', 'resnet18', 'resnet34',
           'resnet50', 'resnet101', 'resnet152', 'get_model']


def _conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def _conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _downsample(ds, x):
    """The projection shortcut (1x1 conv + BatchNorm, no ReLU)."""
    if isinstance(ds, nn.Sequential) and len(ds) == 2 and isinstance(ds[1], nn.BatchNorm2d):
        return bn_act(ds[0](x), ds[1], relu=False)
    return ds(x)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(cin, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        identity = x if self.downsample is None else _downsample(self.downsample, x)
        out = bn_act(self.conv1(x), self.bn1)
        return bn_act(self.conv2(out), self.bn2, relu=True, z=identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv1x1(cin, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = _conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = _conv1x1(planes, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        identity = x if self.downsample is None else _downsample(self.downsample, x)
        out = bn_act(self.conv1(x), self.bn1)
        out = bn_act(self.conv2(out), self.bn2)
        return bn_act(self.conv3(out), self.bn3, relu=True, z=identity)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, zero_init_residual=False, width=64):
        super().__init__()
        w = width
        self.inplanes = w
        self.conv1 = nn.Conv2d(3, w, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(w)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, w, layers[0])
        self.layer2 = self._make_layer(block, 2 * w, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 4 * w, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 8 * w, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(8 * w * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                _conv1x1(self.inplanes, planes * block.expansion, stride),
                nn.BatchNorm2d(planes * block.expansion))
        mods = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            mods.append(block(self.inplanes, planes))
        return nn.Sequential(*mods)

    def forward(self, x):
        return self.forward_top(self.forward_bottom(x))

    # the two halves of the network for a backward split at the layer2 /
    # layer3 boundary (parallel/overlap.py): the top half holds ~90% of the
    # parameters, whose gradients are complete first in backward
    def forward_bottom(self, x):
        x = self.maxpool(bn_act(self.conv1(x), self.bn1))
        return self.layer2(self.layer1(x))

    def forward_top(self, x):
        x = self.layer4(self.layer3(x))
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def split_parameters(self):
        """(bottom, top) parameter lists of forward_bottom / forward_top."""
        bottom = [self.conv1, self.bn1, self.layer1, self.layer2]
        top = [self.layer3, self.layer4, self.fc]
        return ([p for m in bottom for p in m.parameters()],
                [p for m in top for p in m.parameters()])


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)


def resnet_tiny(**kw):
    """Bottleneck ResNet, one block per stage, width 8: the ResNet-50 layer
    types at test-sized factors (CPU tests of the bench / examples)."""
    kw.setdefault('width', 8)
    return ResNet(Bottleneck, [1, 1, 1, 1], **kw)


_MODELS = {'resnet18': resnet18, 'resnet34': resnet34, 'resnet50': resnet50,
           'resnet101': resnet101, 'resnet152': resnet152, 'resnet_tiny': resnet_tiny}


def get_model(name, **kw):
    try:
        return _MODELS[name.lower()](**kw)
    except KeyError:
        raise ValueError('unknown ImageNet model {}'.format(name))
