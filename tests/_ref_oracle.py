"""Run the READ-ONLY reference K-FAC (/root/reference) in a clean subprocess.

Used by tests/test_reference_oracle.py.  The reference needs one shim to run
on torch 2.x (torch.symeig was removed): symeig -> linalg.eigh(...).contiguous()
(SURVEY.md section 0).  No bytecode is written next to the reference sources.
Prints a torch.save'd blob path with per-step grads and final factors.
"""
import sys
sys.dont_write_bytecode = True
import os, json
import torch

REF = os.environ.get('KFAC_REFERENCE', '/root/reference')


def _symeig(t, eigenvectors=True):
    d, Q = torch.linalg.eigh(t)
    return d, Q.contiguous()


def _cholesky(t, upper=False):
    return torch.linalg.cholesky(t, upper=upper)


def main(cfg_path, out_path):
    cfg = json.load(open(cfg_path))
    torch.symeig = _symeig
    torch.cholesky = _cholesky
    sys.path.insert(0, REF)
    import kfac as refkfac
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tests._oracle_common import build_case, run_steps
    model, data = build_case(cfg)
    kw = dict(cfg['kfac'])
    kw['comm_method'] = getattr(refkfac.CommMethod, kw.pop('comm_method', 'COMM_OPT'))
    pre = refkfac.KFAC(model, **kw)
    grads, factors = run_steps(model, pre, data, cfg['steps'])
    torch.save({'grads': grads, 'factors': factors}, out_path)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
