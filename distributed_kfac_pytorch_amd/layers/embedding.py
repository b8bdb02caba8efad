"""Embedding K-FAC layer stub (reference: kfac/layers/embedding.py:7-99).

The reference registers 'embedding' as a known module but its EmbeddingLayer
constructor always raises (embedding.py:20), so any model with nn.Embedding
must pass skip_layers=['embedding'].  Parity: same behaviour here
(SURVEY.md section 7.4 defect #10).  The diagonal-A math the dead code
sketched is kept as `diagonal_factor` for future use.
"""
import torch

from .base import KFACLayer

__all__ = ['EmbeddingLayer', 'diagonal_factor']


class EmbeddingLayer(KFACLayer):
    def __init__(self, *args, **kwargs):
        super(EmbeddingLayer, self).__init__(*args, **kwargs)
        raise ValueError('Embedding layer does not currently work')


def diagonal_factor(indices, num_embeddings):
    """diag(sum_i one_hot(idx_i)^2) / N as a vector of length num_embeddings."""
    flat = indices.reshape(-1).long()
    counts = torch.bincount(flat, minlength=num_embeddings).to(torch.float32)
    return counts / max(1, flat.numel())
