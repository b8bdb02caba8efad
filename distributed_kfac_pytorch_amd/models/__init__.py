"""Model families used by the examples and benchmarks.

resnet         ImageNet ResNet-18/34/50/101/152 (torchvision-equivalent, no torchvision)
resnet_cifar   CIFAR-10 ResNet-20/32/44/56/110/1202 (option-A shortcuts)
lstm_lm        LSTM language model built on kfac.modules.LSTM
transformer_lm decoder-only Transformer LM (BASELINE config #5)
"""
from . import resnet, resnet_cifar, lstm_lm, transformer_lm
from .resnet import resnet50, resnet101, resnet152
from .lstm_lm import LSTMModel
from .transformer_lm import TransformerLM

__all__ = ['resnet', 'resnet_cifar', 'lstm_lm', 'transformer_lm', 'resnet50', 'resnet101',
           'resnet152', 'LSTMModel', 'TransformerLM', 'get_model']


def get_model(name, **kw):
    name = name.lower()
    if name in resnet._MODELS:
        return resnet.get_model(name, **kw)
    if name in resnet_cifar._MODELS:
        return resnet_cifar.get_model(name, **kw)
    raise ValueError('unknown model {}'.format(name))
