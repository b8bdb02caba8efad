"""LSTM built from nn.Linear so K-FAC hooks see every time step.

Parity with kfac/modules/lstm.py:1-225 of the reference (LSTMCellBase,
LSTMCellKFAC, LSTMCell, LSTMLayer, LSTM), with its defects fixed
(SURVEY.md section 7.4 #12): layers > 0 take `hidden_size * directions`
inputs, `batch_first` is honoured, and `permute_hidden` works for packed
sequences.  Each cell's Linear children are registered by K-FAC as
LinearMultiLayer (one factor contribution per time step).
"""
import torch
import torch.nn as nn
from torch.nn.utils.rnn import PackedSequence, pad_packed_sequence, pack_padded_sequence

__all__ = ['LSTMCellBase', 'LSTMCellKFAC', 'LSTMCell', 'LSTMLayer', 'LSTM']


class LSTMCellBase(nn.Module):
    """Abstract cell: forward(input (B, in), (h, c)) -> (h', c')."""

    def __init__(self, input_size, hidden_size, bias=True):
        super(LSTMCellBase, self).__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.bias = bias

    def forward(self, input, hidden):
        raise NotImplementedError

    def extra_repr(self):
        return 'input_size={}, hidden_size={}, bias={}'.format(
            self.input_size, self.hidden_size, self.bias)


class LSTMCellKFAC(LSTMCellBase):
    """One Linear per gate and per source (8 small factors instead of 2 big)."""

    def __init__(self, *args, **kwargs):
        super(LSTMCellKFAC, self).__init__(*args, **kwargs)
        I, H, b = self.input_size, self.hidden_size, self.bias
        for gate in 'ifgo':
            setattr(self, 'linear_{}_i'.format(gate), nn.Linear(I, H, bias=b))
            setattr(self, 'linear_{}_h'.format(gate), nn.Linear(H, H, bias=b))

    def _gate(self, g, x, h):
        return getattr(self, 'linear_{}_i'.format(g))(x) + getattr(self, 'linear_{}_h'.format(g))(h)

    def forward(self, input, hidden):
        h, c = hidden
        i = torch.sigmoid(self._gate('i', input, h))
        f = torch.sigmoid(self._gate('f', input, h))
        g = torch.tanh(self._gate('g', input, h))
        o = torch.sigmoid(self._gate('o', input, h))
        c_next = f * c + i * g
        return o * torch.tanh(c_next), c_next


class LSTMCell(LSTMCellBase):
    """Standard fused-gate cell: two Linears (input->4H, hidden->4H)."""

    def __init__(self, *args, **kwargs):
        super(LSTMCell, self).__init__(*args, **kwargs)
        self.linear_ih = nn.Linear(self.input_size, 4 * self.hidden_size, bias=self.bias)
        self.linear_hh = nn.Linear(self.hidden_size, 4 * self.hidden_size, bias=self.bias)

    def forward(self, input, hidden):
        hx, cx = hidden
        gates = self.linear_ih(input) + self.linear_hh(hx)
        i, f, g, o = gates.chunk(4, 1)
        c_next = torch.sigmoid(f) * cx + torch.sigmoid(i) * torch.tanh(g)
        return torch.sigmoid(o) * torch.tanh(c_next), c_next


class LSTMLayer(nn.Module):
    """Unrolls one cell over the sequence dimension (Python time loop)."""

    def __init__(self, input_size, hidden_size, bias=True, batch_first=False, reverse=False,
                 cell=LSTMCell):
        super(LSTMLayer, self).__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.bias = bias
        self.batch_first = batch_first
        self.reverse = reverse
        self.cell = cell(input_size, hidden_size, bias=bias)
        self.seq_dim = 1 if batch_first else 0

    def forward(self, input, hidden):
        T = input.size(self.seq_dim)
        steps = range(T - 1, -1, -1) if self.reverse else range(T)
        outputs = []
        for t in steps:
            hidden = self.cell(input.select(self.seq_dim, t), hidden)
            outputs.append(hidden[0])
        if self.reverse:
            outputs.reverse()
        return torch.stack(outputs, self.seq_dim), hidden

    def extra_repr(self):
        return 'input_size={}, hidden_size={}, bias={}, batch_first={}, reverse={}'.format(
            self.input_size, self.hidden_size, self.bias, self.batch_first, self.reverse)


def _permute(t, perm):
    return t if perm is None else t.index_select(1, perm)


class LSTM(nn.Module):
    """Multi-layer (optionally bidirectional) LSTM made of LSTMLayers.

    Same call convention as torch.nn.LSTM: input (T, B, I) or (B, T, I) with
    batch_first, optional (h0, c0) of shape (layers*dirs, B, H); returns
    (output, (h_n, c_n)).  PackedSequence inputs are supported.
    """

    def __init__(self, input_size, hidden_size, num_layers=1, bias=True, batch_first=False,
                 dropout=0.0, bidirectional=False, cell=LSTMCell):
        super(LSTM, self).__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.bias = bias
        self.batch_first = batch_first
        self.dropout = dropout
        self.bidirectional = bidirectional
        self.num_directions = 2 if bidirectional else 1
        layers = []
        for i in range(num_layers):
            in_size = input_size if i == 0 else hidden_size * self.num_directions
            dirs = [LSTMLayer(in_size, hidden_size, bias, batch_first, False, cell)]
            if bidirectional:
                dirs.append(LSTMLayer(in_size, hidden_size, bias, batch_first, True, cell))
            layers.append(nn.ModuleList(dirs))
        self.layers = nn.ModuleList(layers)
        self.drop = nn.Dropout(dropout) if dropout > 0 and num_layers > 1 else None

    def permute_hidden(self, hx, permutation):
        if permutation is None:
            return hx
        return _permute(hx[0], permutation), _permute(hx[1], permutation)

    def forward(self, input, hx=None):
        packed = isinstance(input, PackedSequence)
        if packed:
            # unpacking restores the caller's batch order, so hx needs no permutation
            input, lengths = pad_packed_sequence(input, batch_first=self.batch_first)
        batch = input.size(0) if self.batch_first else input.size(1)
        if hx is None:
            z = input.new_zeros(self.num_layers * self.num_directions, batch, self.hidden_size)
            hx = (z, z)
        h_all, c_all = [], []
        x = input
        for i, dirs in enumerate(self.layers):
            outs = []
            for j, layer in enumerate(dirs):
                li = i * self.num_directions + j
                out, (h, c) = layer(x, (hx[0][li], hx[1][li]))
                outs.append(out)
                h_all.append(h)
                c_all.append(c)
            x = torch.cat(outs, -1) if len(outs) > 1 else outs[0]
            if self.drop is not None and i < self.num_layers - 1:
                x = self.drop(x)
        hidden = (torch.stack(h_all), torch.stack(c_all))
        if packed:
            x = pack_padded_sequence(x, lengths, batch_first=self.batch_first,
                                     enforce_sorted=False)
        return x, hidden
