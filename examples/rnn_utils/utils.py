"""BPTT batching and a sharding sampler for the language-model example.

Reference behaviour: examples/rnn_utils/utils.py:7-73 (a DistributedSampler
wrapping a batch sampler) and the BPTT sampler of torchnlp used by
examples/torch_language_model.py:124-164 -- re-implemented without torchnlp.
"""
import math

import torch
from torch.utils.data.sampler import Sampler

__all__ = ['DistributedSampler', 'batchify', 'bptt_batches', 'Corpus']


class DistributedSampler(Sampler):
    """Restrict a sampler (or any sized iterable of indices/batches) to this
    rank's strided shard: rank r gets items r, r + W, r + 2W, ..."""

    def __init__(self, sampler, num_replicas=None, rank=None, shuffle=True):
        import torch.distributed as dist
        if num_replicas is None or rank is None:
            if not dist.is_initialized():
                raise RuntimeError('Requires `torch.distributed` to be initialized.')
            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        if rank >= num_replicas:
            raise IndexError('`rank` must be smaller than the `num_replicas`.')
        self.sampler, self.num_replicas, self.rank, self.shuffle = \
            sampler, num_replicas, rank, shuffle
        self.epoch = 0
        self.num_samples = int(math.ceil(len(self.sampler) / self.num_replicas))
        self.total_size = self.num_samples * self.num_replicas

    def __iter__(self):
        items = list(self.sampler)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.epoch)
            items = [items[i] for i in torch.randperm(len(items), generator=g).tolist()]
        items += items[:(self.total_size - len(items))]
        return iter(items[self.rank:self.total_size:self.num_replicas])

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch):
        self.epoch = epoch


class Corpus(object):
    """Word-level corpus from plain-text train/valid/test files (PTB and
    WikiText-2 layout: `ptb.train.txt` or `wiki.train.tokens`), or a synthetic
    token stream (Zipf-distributed ids) when no files are present."""

    def __init__(self, data_dir=None, dataset='penntreebank', synthetic_tokens=200000,
                 vocab=10000, seed=0):
        names = {'penntreebank': ('ptb.train.txt', 'ptb.valid.txt', 'ptb.test.txt'),
                 'wikitext2': ('wiki.train.tokens', 'wiki.valid.tokens', 'wiki.test.tokens')}
        files = None
        if data_dir is not None:
            cand = [os_path_join(data_dir, n) for n in names.get(dataset, ())]
            if cand and all(_exists(c) for c in cand):
                files = cand
        if files is not None:
            self.dictionary = {}
            self.train, self.valid, self.test = (self._tokenize(f) for f in files)
            self.ntokens = len(self.dictionary)
        else:
            g = torch.Generator().manual_seed(seed)
            ranks = torch.arange(1, vocab + 1, dtype=torch.float64)
            probs = (1.0 / ranks) / (1.0 / ranks).sum()
            def draw(n):
                return torch.multinomial(probs, n, replacement=True, generator=g)
            self.train = draw(synthetic_tokens)
            self.valid = draw(max(synthetic_tokens // 10, 1))
            self.test = draw(max(synthetic_tokens // 10, 1))
            self.ntokens = vocab

    def _tokenize(self, path):
        ids = []
        with open(path, encoding='utf8') as f:
            for line in f:
                for w in line.split() + ['<eos>']:
                    if w not in self.dictionary:
                        self.dictionary[w] = len(self.dictionary)
                    ids.append(self.dictionary[w])
        return torch.tensor(ids, dtype=torch.long)


def os_path_join(a, b):
    import os
    return os.path.join(a, b)


def _exists(p):
    import os
    return os.path.exists(p)


def batchify(data, bsz):
    """1-D token stream -> (T, bsz) columns (trailing tokens dropped)."""
    nbatch = data.size(0) // bsz
    return data[:nbatch * bsz].view(bsz, -1).t().contiguous()


def bptt_batches(source, bptt):
    """Start offsets of the BPTT windows of a batchified source."""
    return list(range(0, source.size(0) - 1, bptt))
