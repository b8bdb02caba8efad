"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel family:
sum of each counter over the dispatches of the K-FAC hand-written kernels (and
the largest library kernels), plus derived ratios.

    python scripts/pmc_summary.py pass1.csv [pass2.csv ...] > summary.txt
"""
import collections
import csv
import re
import sys

FAMILIES = [
    ('pgemm (fused preconditioning chain)', r'pgemm_kernel'),
    ('factor SYRK (implicit im2col)', r'syrk|factor'),
    ('tridiag reduction: symv', r'sytrd_symv'),
    ('tridiag reduction: w', r'sytrd_w_kernel'),
    ('tridiag reduction: x', r'sytrd_x_kernel'),
    ('tridiag reduction: panel update', r'sytrd_update|sytrd_rank'),
    ('Jacobi small-n eigensolver', r'jacobi'),
    ('gather / apply / KL', r'gather_grad|apply_grad|kl_dot|split_copy'),
    ('rocSOLVER', r'rocsolver'),
    ('MIOpen / CK conv', r'igemm|conv|ck::'),
    ('MIOpen batchnorm', r'BatchNorm'),
]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return None


def main(paths):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                name = row.get('Kernel_Name', '')
                fam = family(name)
                if fam is None:
                    continue
                tot[fam][row['Counter_Name']] += float(row['Counter_Value'])
                disp[fam].add((p, row.get('Dispatch_Id')))
    for fam, _ in FAMILIES:
        if fam not in tot:
            continue
        c = tot[fam]
        print('== {}  ({} dispatch records)'.format(fam, len(disp[fam])))
        for k in sorted(c):
            print('   {:28s} {:.4g}'.format(k, c[k]))
        if c.get('SQ_LDS_BANK_CONFLICT') is not None and c.get('SQ_LDS_IDX_ACTIVE'):
            print('   -> LDS bank-conflict cycles / LDS active: {:.3f}'.format(
                c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']))
        hit, miss = c.get('TCC_HIT_sum'), c.get('TCC_MISS_sum')
        if hit is not None and miss is not None and hit + miss > 0:
            print('   -> L2 hit rate: {:.3f}'.format(hit / (hit + miss)))
        if c.get('SQ_BUSY_CYCLES') and c.get('SQ_WAVE_CYCLES'):
            print('   -> wave cycles / busy cycles: {:.1f}'.format(
                c['SQ_WAVE_CYCLES'] / c['SQ_BUSY_CYCLES']))


if __name__ == '__main__':
    main(sys.argv[1:])
