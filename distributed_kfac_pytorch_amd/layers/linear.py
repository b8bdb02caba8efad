"""K-FAC layers for nn.Linear (reference: kfac/layers/linear.py:7-59).

`LinearLayer`: A = a^T a / rows with a bias column of ones, G = g^T g / rows,
where (B, ..., D) hook tensors are flattened to (rows, D) so (B, T, D)
Transformer activations fold T into the SYRK row dimension.
`LinearMultiLayer`: a module called once per time step (LSTM cells): the
factor is the SUM of per-call covariances, each normalised by its own rows.
"""
from . import utils as lutils
from .base import KFACLayer
from ..ops import factors as factor_ops

__all__ = ['LinearLayer', 'LinearMultiLayer']


def _rows2d(x):
    return x.reshape(-1, x.shape[-1])


class LinearLayer(KFACLayer):
    def __init__(self, *args, **kwargs):
        super(LinearLayer, self).__init__(*args, **kwargs)
        self.has_bias = self.module.bias is not None

    def _get_A_factor(self, a_inputs):
        a = lutils.reshape_data(a_inputs, batch_first=self.batch_first, collapse_dims=True)
        if self.has_bias:
            a = lutils.append_bias_ones(a)
        return lutils.get_cov(a)

    def _get_G_factor(self, g_outputs):
        g = lutils.reshape_data(g_outputs, batch_first=self.batch_first, collapse_dims=True)
        return lutils.get_cov(g)

    def _sources(self, tensors, has_bias):
        mats = [_rows2d(t) for t in tensors]
        total = sum(m.shape[0] for m in mats)
        srcs = []
        for m in mats:
            s = factor_ops.linear_source(m, has_bias)
            s.scale = 1.0 / total
            srcs.append(s)
        return srcs

    def _a_sources(self, a_inputs):
        return self._sources(a_inputs, self.has_bias)

    def _g_sources(self, g_outputs):
        return self._sources(g_outputs, False)

    def _g_rows(self, g):
        return _rows2d(g).shape[0]


class LinearMultiLayer(LinearLayer):
    """Linear module invoked several times per step (e.g. per RNN time step)."""

    def _get_A_factor(self, a_inputs):
        total = None
        for a in a_inputs:
            f = super(LinearMultiLayer, self)._get_A_factor([a])
            total = f if total is None else total + f
        return total

    def _get_G_factor(self, g_outputs):
        total = None
        for g in g_outputs:
            f = super(LinearMultiLayer, self)._get_G_factor([g])
            total = f if total is None else total + f
        return total

    def _sources(self, tensors, has_bias):
        srcs = []
        for t in tensors:
            m = _rows2d(t)
            s = factor_ops.linear_source(m, has_bias)
            s.scale = 1.0 / m.shape[0]
            srcs.append(s)
        return srcs

    def _g_rows(self, g):
        return None     # each time step's covariance is normalised on its own
