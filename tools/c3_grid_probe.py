#!/usr/bin/env python3
"""Config-3 grid parity (tests/grid_parity.c3_training_step) under summation-order variants of the generator path, to
see which order change moves a near-cancelling quantity: base; cem_generic (the CEM adjoints on the generic per-output
loop, flags bit 1); fold_einsum (the upsampler phases folded by the round-3 einsum instead of the summed gather).
    usage: python tools/c3_grid_probe.py PRECISION [variant ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'tests'), os.path.join(REPO, 'explorable-super-resolution_old_amd')):
    sys.path.insert(0, p)

import torch  # noqa: E402

import grid_parity as GP  # noqa: E402
from esr_amd import _lib, engine as E  # noqa: E402


def einsum_fold(w, py, px, f=2):
    Fy = torch.tensor(E._FOLDS[f][py][0], dtype=w.dtype, device=w.device)
    Fx = torch.tensor(E._FOLDS[f][px][0], dtype=w.dtype, device=w.device)
    return torch.einsum('ay,bx,oiyx->oiab', Fy, Fx, w.detach())


def f64_fold(w, py, px, f=2):
    t = E.fold_term_images(w.detach().double(), py, px, f)
    return (((t[0] + t[1]) + t[2]) + t[3]).float()


def main():
    prec = sys.argv[1]
    dev = torch.device('cuda', 0)
    lib = _lib.load()
    adj = lib.esr_cem_adjoint
    refresh = E._Packed.refresh
    for name in sys.argv[2:] or ['base']:
        opts = name.split('+')
        if 'cem_generic' in opts:
            lib.esr_cem_adjoint = lambda *a: adj(*(a[:13] + (a[13] | 2,) + a[14:]))
        else:
            lib.esr_cem_adjoint = adj

        fold = einsum_fold if 'fold_einsum' in opts else f64_fold

        def fold_refresh(self, fold=fold):
            refresh(self)
            with torch.no_grad():
                for row, (j, f) in zip(self.up, E.up_stages(self.net)):
                    w = self.net.model[j][1].weight
                    for cw, (py, px) in zip(row, [(a, b) for a in range(f) for b in range(f)]):
                        cw.f32.copy_(E.pack_conv_weight(fold(w, py, px, f), list(range(64)), 64))
        E._Packed.refresh = fold_refresh if ('fold_einsum' in opts or 'fold_f64' in opts) else refresh
        r = GP.c3_training_step(dev, prec)
        print('== %s %s ok %s worst %.4f' % (prec, name, r['ok'], r['worst_frac_of_bound']), flush=True)
        for line in r['lines'][:2]:
            print('   ' + line, flush=True)
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
