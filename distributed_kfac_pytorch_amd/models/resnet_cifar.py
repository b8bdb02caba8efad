"""CIFAR-10 ResNets (He et al. 2016, option-A identity shortcuts).

Same architectures and parameter counts as the reference's
examples/cnn_utils/cifar_resnet.py:40-174 (ResNet-20/32/44/56/110/1202:
0.27M ... 19.4M params), written independently here.  The option-A shortcut
(strided subsampling + zero channel padding) has no parameters, so the
K-FAC layer set is exactly the 3x3 convolutions + the final Linear.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ['CifarResNet', 'resnet20', 'resnet32', 'resnet44', 'resnet56', 'resnet110',
           'resnet1202', 'get_model']


class _PadShortcut(nn.Module):
    """Option A: x[:, :, ::2, ::2] zero-padded to `planes` channels."""

    def __init__(self, planes):
        super().__init__()
        self.pad = planes // 4

    def forward(self, x):
        return F.pad(x[:, :, ::2, ::2], (0, 0, 0, 0, self.pad, self.pad))


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        if stride != 1 or in_planes != planes:
            self.shortcut = _PadShortcut(planes)
        else:
            self.shortcut = nn.Sequential()

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + self.shortcut(x))


class CifarResNet(nn.Module):
    def __init__(self, num_blocks, num_classes=10):
        super().__init__()
        self.in_planes = 16
        self.conv1 = nn.Conv2d(3, 16, 3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(16)
        self.layer1 = self._make_layer(16, num_blocks[0], 1)
        self.layer2 = self._make_layer(32, num_blocks[1], 2)
        self.layer3 = self._make_layer(64, num_blocks[2], 2)
        self.linear = nn.Linear(64, num_classes)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.kaiming_normal_(m.weight)

    def _make_layer(self, planes, n, stride):
        blocks = []
        for s in [stride] + [1] * (n - 1):
            blocks.append(BasicBlock(self.in_planes, planes, s))
            self.in_planes = planes
        return nn.Sequential(*blocks)

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.layer3(self.layer2(self.layer1(out)))
        out = F.avg_pool2d(out, out.size()[3])
        return self.linear(out.view(out.size(0), -1))


def resnet20(**kw):
    return CifarResNet([3, 3, 3], **kw)


def resnet32(**kw):
    return CifarResNet([5, 5, 5], **kw)


def resnet44(**kw):
    return CifarResNet([7, 7, 7], **kw)


def resnet56(**kw):
    return CifarResNet([9, 9, 9], **kw)


def resnet110(**kw):
    return CifarResNet([18, 18, 18], **kw)


def resnet1202(**kw):
    return CifarResNet([200, 200, 200], **kw)


_MODELS = {'resnet20': resnet20, 'resnet32': resnet32, 'resnet44': resnet44,
           'resnet56': resnet56, 'resnet110': resnet110, 'resnet1202': resnet1202}


def get_model(name, **kw):
    try:
        return _MODELS[name.lower()](**kw)
    except KeyError:
        raise ValueError('unknown CIFAR model {}'.format(name))
