"""Layer registry: nn.Module -> K-FAC layer object(s).

Reference: kfac/layers/__init__.py:9-40.  An LSTM cell built from
nn.Linear children maps to one LinearMultiLayer per child.
"""
import torch.nn as nn

from .base import KFACLayer
from .conv import Conv2dLayer
from .embedding import EmbeddingLayer
from .linear import LinearLayer, LinearMultiLayer

__all__ = ['KNOWN_MODULES', 'get_kfac_layers', 'module_requires_grad', 'KFACLayer',
           'Conv2dLayer', 'LinearLayer', 'LinearMultiLayer', 'EmbeddingLayer']

KNOWN_MODULES = {'linear', 'conv2d', 'embedding', 'lstmcell'}


def get_kfac_layers(module, **kwargs):
    """-> list of (module, KFACLayer) pairs for `module`."""
    from .. import modules as km
    if isinstance(module, nn.Linear):
        return [(module, LinearLayer(module, **kwargs))]
    if isinstance(module, nn.Conv2d):
        return [(module, Conv2dLayer(module, **kwargs))]
    if isinstance(module, nn.Embedding):
        return [(module, EmbeddingLayer(module, **kwargs))]
    if isinstance(module, km.LSTMCellBase):
        return [(m, LinearMultiLayer(m, **kwargs)) for m in module.children()]
    if isinstance(module, nn.RNNCellBase):
        raise TypeError('KFAC does not support torch.nn.{RNN,LSTM}Cell. Use '
                        'kfac.modules.{RNN,LSTM}Cell instead for KFAC support.')
    raise NotImplementedError('KFAC does not support layer {}'.format(
        module.__class__.__name__))


def module_requires_grad(module):
    """False if any parameter of `module` has requires_grad=False."""
    return all(p.requires_grad for p in module.parameters())
