import sys, torch
sys.path.insert(0, '/root/repo/explorable-super-resolution_old_amd')
sys.path.insert(0, '.')
sys.path.insert(0, 'explorable-super-resolution_old_amd')
from esr_amd import engine as E
dev = torch.device('cuda', 0)
g = torch.Generator().manual_seed(5)
w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).to(dev)
for py in (0, 1):
    for px in (0, 1):
        Fy = torch.tensor(E._FOLDS[2][py][0], dtype=w.dtype, device=dev)
        Fx = torch.tensor(E._FOLDS[2][px][0], dtype=w.dtype, device=dev)
        ein = torch.einsum('ay,bx,oiyx->oiab', Fy, Fx, w)
        terms = E.fold_terms(py, px)
        for a in range(2):
            for b in range(2):
                tt = terms[a][b]
                if len(tt) != 4:
                    continue
                t = [w[:, :, y, x] for (y, x) in tt]
                cands = {'seq': ((t[0] + t[1]) + t[2]) + t[3], 'pair': (t[0] + t[1]) + (t[2] + t[3]),
                         'colpair': (t[0] + t[2]) + (t[1] + t[3]), 'colseq': ((t[0] + t[2]) + t[1]) + t[3],
                         'rev': ((t[3] + t[2]) + t[1]) + t[0], 'revpair': (t[3] + t[2]) + (t[1] + t[0])}
                e = ein[:, :, a, b]
                print(py, px, a, b, tt, {k: int((v != e).sum()) for k, v in cands.items()})
