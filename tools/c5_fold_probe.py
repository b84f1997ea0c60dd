#!/usr/bin/env python3
"""Config-5 grid parity lines (tests/grid_parity.c5_z_gradients) with the upsampler phase weights folded as the packed
gather sums them (default) and, for comparison, as the round-3 einsum fold (a GEMM over 0/1 fold matrices): whether
the fold's summation order moves the C5 margins.    usage: python tools/c5_fold_probe.py [kernel]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'tests'), os.path.join(REPO, 'explorable-super-resolution_old_amd')):
    sys.path.insert(0, p)

import torch  # noqa: E402

import grid_parity as GP  # noqa: E402
from esr_amd import engine as E  # noqa: E402


def einsum_fold(w, py, px, f=2):
    Fy = torch.tensor(E._FOLDS[f][py][0], dtype=w.dtype, device=w.device)
    Fx = torch.tensor(E._FOLDS[f][px][0], dtype=w.dtype, device=w.device)
    return torch.einsum('ay,bx,oiyx->oiab', Fy, Fx, w.detach())


def main():
    kernel = sys.argv[1] if len(sys.argv) > 1 else 'learned13'
    dev = torch.device('cuda', 0)
    r = GP.c5_z_gradients(dev, 'x3', kernel)
    print('== summed-gather fold: worst %.4f' % r['worst_frac_of_bound'])
    print('\n'.join('   ' + l for l in r['lines']))
    orig = E._Packed.train_x3

    def patched(self):
        if not getattr(self, '_einsum_done', False):
            self._einsum_done = True
            with torch.no_grad():
                for row, (j, f) in zip(self.up, E.up_stages(self.net)):
                    w = self.net.model[j][1].weight
                    for cw, (py, px) in zip(row, [(a, b) for a in range(f) for b in range(f)]):
                        new = E.pack_conv_weight(einsum_fold(w, py, px, f), list(range(64)), 64)
                        print('   up %d (%d,%d): max |einsum - summed| %.3e' % (j, py, px,
                                                                             float((new - cw.f32).abs().max())))
                        cw.f32.copy_(new)
            self.version = getattr(self, 'version', 0) + 1
        return orig(self)
    E._Packed.train_x3 = patched
    r = GP.c5_z_gradients(dev, 'x3', kernel)
    print('== einsum fold: worst %.4f' % r['worst_frac_of_bound'])
    print('\n'.join('   ' + l for l in r['lines']))


if __name__ == '__main__':
    main()
