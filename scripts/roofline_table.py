"""Roofline table (profiles/README.md) from rocprofv3 outputs of
scripts/probes/probe_roofline.py: kernel-trace stats (durations) + PMC passes
(MFMA ops, MFMA busy, LDS, FETCH_SIZE, WRITE_SIZE), matched by kernel name.

Conventions (guide: MI355X_MICROARCH.md): FLOPs = 512 x SQ_INSTS_VALU_MFMA_MOPS_*;
FETCH_SIZE / WRITE_SIZE in KiB at the L2's fabric side (Infinity-Cache hits
included; FETCH_SIZE counts wide streaming reads at half their bytes, so the
fetched-bytes column doubles it); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over
1024 SIMDs x 2.42 GHz x kernel time.  Peaks: f32 MFMA 157.3 TF/s, bf16 MFMA
2.5 PF/s dense, HBM 8 TB/s."""
import csv
import sys
from collections import defaultdict

CLK, SIMDS = 2.42e9, 1024


def load_pmc(path):
    d = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d[r['kernel']][r['counter']] = float(r['sum'])
    return d


def main(stats, mfma, fetch, write, keys):
    dur = {}
    for r in csv.DictReader(open(stats)):
        dur[r['Name'][:90]] = (int(r['Calls']), float(r['TotalDurationNs']) * 1e-9)
    m, f, w = load_pmc(mfma), load_pmc(fetch), load_pmc(write)
    print('| kernel | calls | ms | TF/s | % peak | MFMA busy | fetched GB/s | written GB/s | '
          'LDS conflict cycles / LDS cycles |')
    print('|---|---|---|---|---|---|---|---|---|')
    for key, label in keys:
        name = next((k for k in dur if key in k), None)
        if name is None:
            continue
        calls, t = dur[name]
        mm = next((v for k, v in m.items() if key in k), {})
        ff = next((v for k, v in f.items() if key in k), {})
        ww = next((v for k, v in w.items() if key in k), {})
        f32 = mm.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0) * 512
        b16 = mm.get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0) * 512
        flops, peak = (f32, 157.3e12) if f32 >= b16 else (b16, 2.5e15)
        busy = mm.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (SIMDS * CLK * t)
        fb = 2 * ff.get('FETCH_SIZE', 0) * 1024 / t / 1e9
        wb = ww.get('WRITE_SIZE', 0) * 1024 / t / 1e9
        lds = mm.get('SQ_LDS_IDX_ACTIVE', 0)
        conf = ('%.0f %%' % (100 * mm.get('SQ_LDS_BANK_CONFLICT', 0) / lds)) if lds else '-'
        tf = ('%.1f' % (flops / t / 1e12)) if flops else '-'
        pk = ('%.0f %%' % (100 * flops / t / peak)) if flops else '-'
        bz = ('%.0f %%' % (100 * busy)) if mm else '-'
        print('| %s | %d | %.2f | %s | %s | %s | %.0f | %.0f | %s |' % (
            label, calls, t * 1e3, tf, pk, bz, fb, wb, conf))


if __name__ == '__main__':
    KEYS = [('pgemm_kernel<0', 'pgemm fp32 (chain + eigensolver GEMMs)'),
            ('pgemm_kernel<1', 'pgemm bf16x3 (chain)'),
            ('syrk_vec_grouped_kernel<1', 'factor SYRK, grouped (bf16)'),
            ('syrk_patch_kernel', 'factor SYRK, im2col path (first conv)'),
            ('tile_reduce_kernel', 'split-K tile reduce'),
            ('factor_ema_grouped_kernel', 'factor EMA, grouped'),
            ('split_copy_kernel<0', 'eigendata split/copy'),
            ('gather_grad_kernel<0', 'gradient gather'),
            ('sytrd_symv2_kernel', 'reduction: symv'),
            ('sytrd_fin_kernel', 'reduction: column finish'),
            ('sytrd_upd_kernel', 'reduction: panel update')]
    main(*sys.argv[1:5], KEYS)
