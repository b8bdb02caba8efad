"""Regenerate tests/fixtures/training_quality_resnet20.pt: the READ-ONLY
reference K-FAC (/root/reference/kfac, run in a subprocess with its one torch-2
shim, as tests/_ref_oracle.py) training ResNet-20 on the task of
tests/_training_task.py for 100 steps on the CPU, plus an SGD-only run of the
same task for information.  Stored weights-only: per-step losses and the
first step's K-FAC-preconditioned gradients.

    python scripts/make_training_fixture.py [--out PATH]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get('KFAC_REFERENCE', '/root/reference')

_CHILD = r'''
import sys, json
sys.dont_write_bytecode = True
import torch
torch.symeig = lambda t, eigenvectors=True: (lambda d, q: (d, q.contiguous()))(*torch.linalg.eigh(t))
sys.path.insert(0, {ref!r})
sys.path.insert(0, {root!r})
import kfac as refkfac
from tests import _training_task as T
torch.set_num_threads(8)
net = T.model()
data = T.batches()
pre = refkfac.KFAC(net, **T.KFAC_KW)
opt = torch.optim.SGD(net.parameters(), **T.SGD_KW)
losses, grads0 = [], None
for i, (x, y) in enumerate(data):
    opt.zero_grad()
    loss = T.loss_fn(net(x), y)
    loss.backward()
    pre.step()
    if i == 0:
        grads0 = [p.grad.detach().clone() for p in net.parameters()]
    opt.step()
    losses.append(float(loss))
torch.save({{'losses': torch.tensor(losses, dtype=torch.float64), 'grads0': grads0}}, {out!r})
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default=os.path.join(ROOT, 'tests', 'fixtures',
                                                  'training_quality_resnet20.pt'))
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    import torch
    from tests import _training_task as T
    with tempfile.TemporaryDirectory() as td:
        blob = os.path.join(td, 'ref.pt')
        code = _CHILD.format(ref=REF, root=ROOT, out=blob)
        r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True,
                           env=dict(os.environ, PYTHONDONTWRITEBYTECODE='1'))
        if r.returncode != 0:
            raise SystemExit(r.stderr[-3000:])
        ref = torch.load(blob, weights_only=True)
    torch.set_num_threads(8)
    sgd = T.run_eager(T.model(), None, T.batches())
    cfg = dict(steps=T.STEPS, batch=T.BATCH, snr=T.SNR, kfac=T.KFAC_KW, sgd=T.SGD_KW,
               source='reference kfac/ (CPU, fp32), scripts/make_training_fixture.py')
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    torch.save({'losses': ref['losses'], 'grads0': ref['grads0'],
                'sgd_losses': torch.tensor(sgd, dtype=torch.float64),
                'config': json.dumps(cfg)}, args.out)
    km, sm = T.window_means(ref['losses'].tolist()), T.window_means(sgd)
    print('reference K-FAC loss, 25-step windows:', ' '.join('%.4f' % v for v in km))
    print('SGD only            , 25-step windows:', ' '.join('%.4f' % v for v in sm))
    print('step 100: K-FAC %.4f  SGD %.4f' % (ref['losses'][-1], sgd[-1]))
    print('wrote', args.out)


if __name__ == '__main__':
    main()
