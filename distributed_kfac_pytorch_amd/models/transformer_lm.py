"""Decoder-only Transformer LM for the K-FAC HYBRID_OPT language-model config.

BASELINE.json config #5 names a "Transformer LM" for the language-model
example (the reference itself only ships an LSTM LM).  Every projection is an
nn.Linear on (B, T, D) activations, so each K-FAC Linear factor folds B*T into
the SYRK row dimension (layers/linear.py); attention uses
F.scaled_dot_product_attention.  K-FAC skips the embedding
(`skip_layers=['embedding']`); LayerNorm is not a K-FAC module.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ['TransformerLM', 'Block']


class Block(nn.Module):
    def __init__(self, d_model, n_heads, d_ff, dropout=0.0):
        super().__init__()
        self.n_heads = n_heads
        self.ln1 = nn.LayerNorm(d_model)
        self.qkv = nn.Linear(d_model, 3 * d_model)
        self.proj = nn.Linear(d_model, d_model)
        self.ln2 = nn.LayerNorm(d_model)
        self.fc1 = nn.Linear(d_model, d_ff)
        self.fc2 = nn.Linear(d_ff, d_model)
        self.dropout = dropout

    def forward(self, x):
        B, T, D = x.shape
        h = self.ln1(x)
        q, k, v = self.qkv(h).view(B, T, 3, self.n_heads, D // self.n_heads).unbind(2)
        q, k, v = (t.transpose(1, 2) for t in (q, k, v))
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True,
                                           dropout_p=self.dropout if self.training else 0.0)
        x = x + self.proj(a.transpose(1, 2).reshape(B, T, D))
        x = x + self.fc2(F.gelu(self.fc1(self.ln2(x))))
        return x


class TransformerLM(nn.Module):
    def __init__(self, vocab, d_model=512, n_layers=6, n_heads=8, d_ff=2048, max_len=1024,
                 dropout=0.0):
        super().__init__()
        self.tok = nn.Embedding(vocab, d_model)
        self.pos = nn.Embedding(max_len, d_model)
        self.blocks = nn.ModuleList([Block(d_model, n_heads, d_ff, dropout)
                                     for _ in range(n_layers)])
        self.ln_f = nn.LayerNorm(d_model)
        self.head = nn.Linear(d_model, vocab, bias=False)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, std=0.02)
        for b in self.blocks:
            nn.init.normal_(b.proj.weight, std=0.02 / math.sqrt(2 * n_layers))
            nn.init.normal_(b.fc2.weight, std=0.02 / math.sqrt(2 * n_layers))

    def forward(self, idx):
        B, T = idx.shape
        pos = torch.arange(T, device=idx.device)
        x = self.tok(idx) + self.pos(pos)[None]
        for b in self.blocks:
            x = b(x)
        return self.head(self.ln_f(x))
