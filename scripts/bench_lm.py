"""Language-model K-FAC throughput: this framework vs the READ-ONLY reference.

The reference's language-model example (examples/torch_language_model.py:
239-300, examples/rnn_utils/lstm.py:14-63, examples/cnn_utils/optimizers.py:
8-45) trains a 2-layer 650-unit LSTM on Penn Treebank with K-FAC:
bptt 35, batch 20, factors every step, eigendecompositions every 10,
damping 2e-3, factor decay 0.95, kl_clip 1e-3, skip_layers
['linear', 'embedding'] (only the LSTM gate cells are preconditioned),
dropout 0.5, gradient clipping 0.25, torch DDP.  This script times that
training step on one GPU (synthetic token stream of the PTB vocabulary size,
no dataset in the image) for

    --impl ours       distributed_kfac_pytorch_amd (LSTMModel + KFAC, fp32 preconditioning)
    --impl reference  the reference kfac + its LSTMModel, imported from the
                      extracted reference tree (torch.symeig shim as in
                      scripts/bench_reference.py)

and also `--model transformer` (ours only: BASELINE.json config #5's
Transformer LM, 6 x 512, HYBRID_OPT).  W warmup steps, the K-FAC step
counter reset so the window opens with an inverse step, device synchronize
on both sides; prints one JSON line (tokens/s over the window, ms by step
kind).

    python scripts/bench_lm.py --impl ours --steps 50 --warmup 10
    python scripts/bench_lm.py --impl reference --ref-tar ref_snapshot/kfac_reference.tar
"""
import argparse
import importlib.util
import json
import os
import sys
import time

sys.dont_write_bytecode = True

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'scripts'))


def build_reference(args, dev):
    from bench_reference import import_reference
    refkfac = import_reference(args.ref_dir, args.ref_tar)
    refkfac.comm.init_comm_backend()
    ref_dir = os.path.dirname(os.path.dirname(os.path.abspath(refkfac.__file__)))
    spec = importlib.util.spec_from_file_location(
        'ref_rnn_lstm', os.path.join(ref_dir, 'examples', 'rnn_utils', 'lstm.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    model = mod.LSTMModel(args.vocab, args.emsize, args.nhid, args.nlayers,
                          dropout=args.dropout, tie_weights=False).to(dev)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.SGD(model.parameters(), lr=args.lr)
    pre = None
    if not args.no_kfac:
        pre = refkfac.KFAC(model, damping=args.damping, factor_decay=0.95,
                           factor_update_freq=args.kfac_cov_update_freq,
                           inv_update_freq=args.kfac_update_freq, kl_clip=0.001, lr=args.lr,
                           batch_first=False, comm_method=getattr(refkfac.CommMethod, args.comm),
                           distribute_layer_factors=True, grad_worker_fraction=0.25,
                           skip_layers=['linear', 'embedding'], use_eigen_decomp=True)

    def fwd(data, hidden):
        if hidden is not None:
            hidden = model.detach(hidden)
        out, hidden = ddp(data, hidden)
        return out, hidden
    return model, opt, pre, fwd, nn.NLLLoss()


def build_ours(args, dev):
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd.models import LSTMModel, TransformerLM
    if args.model == 'lstm':
        model = LSTMModel(args.vocab, args.emsize, args.nhid, args.nlayers, args.dropout).to(dev)
        skip = ['linear', 'embedding']
    else:
        model = TransformerLM(args.vocab, d_model=512, n_layers=6, n_heads=8, d_ff=2048,
                              max_len=max(args.bptt, 64)).to(dev)
        # the 10k-vocabulary head's 10k x 10k gradient factor would dominate
        # the inverse update (the reference's LSTM config skips its decoder
        # the same way, skip_layers=['linear', 'embedding'])
        skip = ['embedding', 'head'] if args.skip_head else ['embedding']
    # one rank + graphs: no DDP wrapper (nothing to all-reduce; the step is
    # captured whole by GraphedTrainStep)
    ddp = model if args.graphs else \
        torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.SGD(model.parameters(), lr=args.lr)
    pre = None
    if not args.no_kfac:
        pre = kfac.KFAC(model, damping=args.damping, factor_decay=0.95,
                        factor_update_freq=args.kfac_cov_update_freq,
                        inv_update_freq=args.kfac_update_freq, kl_clip=0.001, lr=args.lr,
                        comm_method=getattr(kfac.CommMethod, args.comm), grad_worker_fraction=0.25,
                        skip_layers=skip, accumulate_data=args.model == 'lstm',
                        batch_first=False, precond_precision=args.precond_precision)

    def fwd(data, hidden):
        if args.model == 'lstm':
            if hidden is not None:
                hidden = tuple(h.detach() for h in hidden)
            return ddp(data, hidden)
        return ddp(data.t().contiguous()).transpose(0, 1), None
    return model, opt, pre, fwd, nn.CrossEntropyLoss()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--impl', default='ours', choices=['ours', 'reference'])
    ap.add_argument('--model', default='lstm', choices=['lstm', 'transformer'])
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch-size', type=int, default=20)
    ap.add_argument('--bptt', type=int, default=35)
    ap.add_argument('--vocab', type=int, default=10000)
    ap.add_argument('--emsize', type=int, default=650)
    ap.add_argument('--nhid', type=int, default=650)
    ap.add_argument('--nlayers', type=int, default=2)
    ap.add_argument('--dropout', type=float, default=0.5)
    ap.add_argument('--lr', type=float, default=10.0)
    ap.add_argument('--damping', type=float, default=0.002)
    ap.add_argument('--kfac-update-freq', type=int, default=10)
    ap.add_argument('--kfac-cov-update-freq', type=int, default=1)
    ap.add_argument('--precond-precision', default='fp32', choices=['fp32', 'bf16x3', 'bf16x6'])
    ap.add_argument('--no-kfac', action='store_true')
    ap.add_argument('--autocast', default='none', choices=['none', 'bf16'],
                    help='bf16 autocast of forward + loss (both implementations)')
    ap.add_argument('--skip-head', type=int, default=1,
                    help='transformer: leave the vocabulary projection out of K-FAC')
    ap.add_argument('--graphs', type=int, default=0,
                    help='ours, one GPU: capture the whole step (graphs.GraphedTrainStep)')
    ap.add_argument('--ref-dir', default=os.environ.get('KFAC_REFERENCE', '/root/reference'))
    ap.add_argument('--ref-tar', default=None)
    args = ap.parse_args()
    if args.impl == 'reference' and args.model != 'lstm':
        raise SystemExit('the reference ships only the LSTM language model')
    if args.graphs and args.impl == 'reference':
        raise SystemExit('--graphs is this framework\'s GraphedTrainStep')

    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29534')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    dev = torch.device('cuda', int(os.environ.get('LOCAL_RANK', 0)))
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl')
    world = dist.get_world_size()
    torch.manual_seed(1111)
    args.comm = 'HYBRID_OPT'
    if args.impl == 'reference' and world == 1:
        # the reference's HYBRID_OPT computes size % min(1, round(size * fraction))
        # = 1 % 0 at world 1 (kfac/preconditioner.py:246); on one GPU no method
        # communicates, so COMM_OPT times the same work
        args.comm = 'COMM_OPT'
    build = build_reference if args.impl == 'reference' else build_ours
    model, opt, pre, fwd, crit = build(args, dev)

    B, T = args.batch_size, args.bptt
    g = torch.Generator(device=dev).manual_seed(0)
    stream = torch.randint(0, args.vocab, (T * 64 + 1, B), device=dev, generator=g)
    state = {'hidden': None, 'i': 0}

    def step():
        i = state['i']
        state['i'] = (i + T) % (T * 64)
        data, target = stream[i:i + T], stream[i + 1:i + 1 + T].reshape(-1)
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=args.autocast == 'bf16'):
            out, state['hidden'] = fwd(data, state['hidden'])
            loss = crit(out.reshape(-1, out.size(-1)), target)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.25)
        if pre is not None:
            pre.step()
        opt.step()
        return loss

    if args.graphs:
        from distributed_kfac_pytorch_amd import graphs
        # static inputs: each step copies its batch (and the carried LSTM
        # state) into these; the captured step writes the new state back
        x_buf = torch.empty(T, B, dtype=torch.long, device=dev)
        y_buf = torch.empty(T * B, dtype=torch.long, device=dev)
        h_buf = model.init_hidden(B) if args.model == 'lstm' else None

        def body():
            opt.zero_grad(set_to_none=True)
            with torch.autocast('cuda', dtype=torch.bfloat16, enabled=args.autocast == 'bf16'):
                if h_buf is not None:
                    out, hid = model(x_buf, h_buf)
                else:
                    out = model(x_buf.t()).transpose(0, 1)
                loss = crit(out.reshape(-1, out.size(-1)), y_buf)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 0.25)
            if pre is not None:
                pre.step()
            opt.step()
            if h_buf is not None:
                with torch.no_grad():
                    h_buf[0].copy_(hid[0])
                    h_buf[1].copy_(hid[1])
            return loss
        gstep = graphs.GraphedTrainStep(body, pre, [opt])

        def step():     # noqa: F811
            i = state['i']
            state['i'] = (i + T) % (T * 64)
            x_buf.copy_(stream[i:i + T])
            y_buf.copy_(stream[i + 1:i + 1 + T].reshape(-1))
            return gstep()

    for i in range(args.warmup):
        step()
    if pre is not None:
        pre.param_groups[0]['step'] = 0
    f = args.kfac_update_freq
    kinds, evs = [], []
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        kinds.append(('inverse' if i % f == 0 else 'factor') if pre is not None else 'plain')
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        evs.append(e)
        loss = step()
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    evs.append(e)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    per = {}
    for k, a, b in zip(kinds, evs[:-1], evs[1:]):
        per.setdefault(k, []).append(a.elapsed_time(b))
    rec = {'metric': 'tokens/sec %s LM K-FAC+SGD (%s)' % (args.model, args.impl)
                     if pre is not None else 'tokens/sec %s LM SGD (%s)' % (args.model, args.impl),
           'value': round(B * T * world * args.steps / el, 1), 'unit': 'tokens/s',
           'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
           'ms_per_step': round(el / args.steps * 1e3, 3),
           'step_ms_by_kind': {k: round(sum(v) / len(v), 3) for k, v in per.items()},
           'steps_by_kind': {k: len(v) for k, v in per.items()},
           'final_loss': round(float(loss.item()), 4),
           'config': {'batch': B, 'bptt': T, 'vocab': args.vocab,
                      **({'emsize': args.emsize, 'nhid': args.nhid, 'nlayers': args.nlayers}
                         if args.model == 'lstm' else
                         {'d_model': 512, 'n_layers': 6, 'n_heads': 8, 'd_ff': 2048,
                          'kfac_skips_head': bool(args.skip_head)}),
                      'comm_method': args.comm, 'graphs': bool(args.graphs),
                      'autocast': args.autocast, 'inv_update_freq': f, 'factor_update_freq': args.kfac_cov_update_freq,
                      'precond_precision': args.precond_precision if args.impl == 'ours' else 'fp32'},
           'data': 'synthetic'}
    if dist.get_rank() == 0:
        print(json.dumps(rec), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
