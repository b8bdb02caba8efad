"""Language model + K-FAC: LSTM (reference parity) or Transformer (BASELINE config #5).

Reference: examples/torch_language_model.py (LSTM on PTB / WikiText-2 through
torchnlp).  The reference script is broken as shipped (SURVEY.md 7.4 #13:
`base_lr = rank * world`, a 4-value unpack of a 3-tuple, missing CLI args);
this is a working rewrite of its behaviour:

  * data: plain-text PTB / WikiText-2 files under --data-dir, else a synthetic
    Zipf token stream; batchify per rank (each rank takes its own columns),
    BPTT windows of --bptt tokens;
  * model: `--model lstm` = Embedding -> kfac.modules.LSTM -> Linear
    (optionally tied); `--model transformer` = decoder-only Transformer;
  * K-FAC skips the embedding (its layer type is unsupported, as in the
    reference) and, with --tied, the decoder too (the reference's
    --register-tied path fed integer token ids into a Linear factor and
    cannot work; the tied weight gets plain SGD gradients);
  * HYBRID_OPT with grad_worker_fraction 0.25 is the BASELINE LM config.

Launch: python -m torch.distributed.run --nproc-per-node 8 --master-addr
127.0.0.1 examples/torch_language_model.py --model transformer ...
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import LSTMModel, TransformerLM  # noqa: E402
from distributed_kfac_pytorch_amd.parallel import launch  # noqa: E402
from examples.rnn_utils.utils import Corpus, batchify, bptt_batches  # noqa: E402
from examples.utils import Metric  # noqa: E402

COMM = {'comm-opt': kfac.CommMethod.COMM_OPT, 'mem-opt': kfac.CommMethod.MEM_OPT,
        'hybrid-opt': kfac.CommMethod.HYBRID_OPT}


def parse(argv=None):
    p = argparse.ArgumentParser(description='LM + K-FAC',
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument('--data-dir', default=None)
    p.add_argument('--dataset', default='penntreebank', choices=['penntreebank', 'wikitext2'])
    p.add_argument('--synthetic-tokens', type=int, default=200000)
    p.add_argument('--vocab', type=int, default=10000, help='synthetic vocabulary size')
    p.add_argument('--log-dir', default='./logs')
    p.add_argument('--model', default='lstm', choices=['lstm', 'transformer'])
    p.add_argument('--emsize', type=int, default=650)
    p.add_argument('--nhid', type=int, default=650)
    p.add_argument('--nlayers', type=int, default=2)
    p.add_argument('--nheads', type=int, default=8)
    p.add_argument('--bptt', type=int, default=35)
    p.add_argument('--dropout', type=float, default=0.5)
    p.add_argument('--tied', action='store_true')
    p.add_argument('--batch-size', type=int, default=20)
    p.add_argument('--eval-batch-size', type=int, default=10)
    p.add_argument('--epochs', type=int, default=40)
    p.add_argument('--base-lr', type=float, default=10.0)
    p.add_argument('--lr-decay-epoch', type=int, default=1000)
    p.add_argument('--lr-decay-rate', type=float, default=1 / 1.2)
    p.add_argument('--clip', type=float, default=0.25)
    p.add_argument('--seed', type=int, default=1111)
    p.add_argument('--no-cuda', action='store_true')
    p.add_argument('--kfac-update-freq', type=int, default=10)
    p.add_argument('--kfac-cov-update-freq', type=int, default=1)
    p.add_argument('--stat-decay', type=float, default=0.95)
    p.add_argument('--damping', type=float, default=0.002)
    p.add_argument('--kl-clip', type=float, default=0.001)
    p.add_argument('--skip-layers', nargs='+', default=['embedding'])
    p.add_argument('--kfac-comm-method', default='hybrid-opt', choices=sorted(COMM))
    p.add_argument('--kfac-grad-worker-fraction', type=float, default=0.25)
    p.add_argument('--precond-precision', default='bf16x6', choices=['bf16x6', 'fp32', 'bf16x3'],
                   help='preconditioning GEMMs: bf16x6 = six bf16 MFMA products per fp32 '
                        'product (fp32-level error), fp32 = exact f32 MFMA, bf16x3 = ~1e-5')
    p.add_argument('--verbose', action='store_true')
    return p.parse_args(argv)


def get_batch(source, i, bptt):
    seq_len = min(bptt, len(source) - 1 - i)
    return source[i:i + seq_len], source[i + 1:i + 1 + seq_len].reshape(-1)


def run_model(model, data, hidden, args):
    if args.model == 'lstm':
        out, hidden = model(data, hidden)
        return out, tuple(h.detach() for h in hidden)
    return model(data.t().contiguous()).transpose(0, 1), None   # (B, T) in, (T, B, V) out


def main(argv=None):
    args = parse(argv)
    device = launch.init_distributed(no_cuda=args.no_cuda)
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    torch.manual_seed(args.seed)

    corpus = Corpus(args.data_dir, args.dataset, args.synthetic_tokens, args.vocab,
                    seed=args.seed)
    # every rank trains on its own columns of the batchified stream
    train = batchify(corpus.train, args.batch_size * world)[:, rank::world].contiguous()
    val = batchify(corpus.valid, args.eval_batch_size)
    train, val = train.to(device), val.to(device)

    if args.model == 'lstm':
        model = LSTMModel(corpus.ntokens, args.emsize, args.nhid, args.nlayers, args.dropout,
                          args.tied)
    else:
        model = TransformerLM(corpus.ntokens, d_model=args.emsize, n_layers=args.nlayers,
                              n_heads=args.nheads, d_ff=4 * args.emsize,
                              max_len=max(args.bptt, 64), dropout=0.0)
    model = model.to(device)
    ddp = launch.wrap_ddp(model, device)

    lr = args.base_lr * world      # the reference wrote rank * world (defect #13)
    optimizer = torch.optim.SGD(model.parameters(), lr=lr)
    skip = list(args.skip_layers)
    if args.tied and args.model == 'lstm':
        skip = skip + ['linear']     # the decoder (LSTM gates register as lstmcell)
    pre = None
    if args.kfac_update_freq > 0:
        pre = kfac.KFAC(model, damping=args.damping, factor_decay=args.stat_decay,
                        factor_update_freq=args.kfac_cov_update_freq,
                        inv_update_freq=args.kfac_update_freq, kl_clip=args.kl_clip, lr=lr,
                        comm_method=COMM[args.kfac_comm_method],
                        grad_worker_fraction=args.kfac_grad_worker_fraction,
                        skip_layers=skip, accumulate_data=args.model == 'lstm',
                        batch_first=False, precond_precision=args.precond_precision,
                        verbose=args.verbose and rank == 0)
    sched = torch.optim.lr_scheduler.StepLR(optimizer, args.lr_decay_epoch, args.lr_decay_rate)
    criterion = nn.CrossEntropyLoss()
    history = []
    for epoch in range(args.epochs):
        model.train()
        t0 = time.time()
        hidden = model.init_hidden(train.size(1)) if args.model == 'lstm' else None
        loss_m = Metric('train_loss')
        for i in bptt_batches(train, args.bptt):
            data, targets = get_batch(train, i, args.bptt)
            optimizer.zero_grad()
            out, hidden = run_model(ddp, data, hidden, args)
            loss = criterion(out.reshape(-1, out.size(-1)), targets)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), args.clip)
            if pre is not None:
                pre.step()
            optimizer.step()
            loss_m.update(loss)
        model.eval()
        val_m = Metric('val_loss')
        with torch.no_grad():
            hidden = model.init_hidden(val.size(1)) if args.model == 'lstm' else None
            for i in bptt_batches(val, args.bptt):
                data, targets = get_batch(val, i, args.bptt)
                out, hidden = run_model(model, data, hidden, args)
                val_m.update(criterion(out.reshape(-1, out.size(-1)), targets))
        sched.step()
        tl, vl = float(loss_m.avg), float(val_m.avg)
        rec = {'epoch': epoch + 1, 'train_loss': tl, 'train_ppl': math.exp(min(tl, 50)),
               'val_loss': vl, 'val_ppl': math.exp(min(vl, 50)), 'time': time.time() - t0}
        history.append(rec)
        if rank == 0:
            print(json.dumps(rec), flush=True)
    return history


if __name__ == '__main__':
    main()
