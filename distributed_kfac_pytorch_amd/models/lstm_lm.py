"""LSTM language model (reference: examples/rnn_utils/lstm.py:14-63).

Embedding -> N x kfac.modules.LSTM -> Linear decoder, optional weight tying.
The LSTM is built from nn.Linear cells so K-FAC registers every gate
projection (LinearMultiLayer: one factor term per time step).  K-FAC must
skip the embedding (`skip_layers=['embedding']`, reference parity) and, when
the decoder is tied, either skip it or use `register_shared_module`.
"""
import torch.nn as nn

from ..modules import LSTM

__all__ = ['LSTMModel']


class LSTMModel(nn.Module):
    def __init__(self, ntoken, ninp, nhid, nlayers, dropout=0.5, tie_weights=False,
                 batch_first=False):
        super().__init__()
        self.drop = nn.Dropout(dropout)
        self.encoder = nn.Embedding(ntoken, ninp)
        self.rnn = LSTM(ninp, nhid, nlayers, dropout=dropout, batch_first=batch_first)
        self.decoder = nn.Linear(nhid, ntoken)
        if tie_weights:
            if nhid != ninp:
                raise ValueError('When using the tied flag, nhid must be equal to emsize')
            self.decoder.weight = self.encoder.weight
        self.nhid, self.nlayers = nhid, nlayers
        self.encoder.weight.data.uniform_(-0.1, 0.1)
        self.decoder.bias.data.zero_()
        self.decoder.weight.data.uniform_(-0.1, 0.1)

    def forward(self, input, hidden=None):
        emb = self.drop(self.encoder(input))
        output, hidden = self.rnn(emb, hidden)
        return self.decoder(self.drop(output)), hidden

    def init_hidden(self, bsz):
        w = next(self.parameters())
        z = w.new_zeros(self.nlayers, bsz, self.nhid)
        return (z, z.clone())
