"""Diagnostics for the production-grid parity checks (tests/grid_parity.py): every failing quantity, untruncated."""
import sys
import os
_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
for _p in (_R, os.path.join(_R, 'explorable-super-resolution_old_amd'), os.path.join(_R, 'tests')):
    sys.path.insert(0, _p)
import torch  # noqa: E402
import grid_parity as GP  # noqa: E402

dev = torch.device('cuda', 0)
which = sys.argv[1:] or ['c3:f32']
for w in which:
    kind, prec = w.split(':')
    r = GP.c3_training_step(dev, prec) if kind == 'c3' else GP.c5_z_gradients(dev, prec)
    print('==', w, 'ok', r['ok'], 'worst', r['worst_frac_of_bound'], flush=True)
    for line in r['lines']:
        print('  ', line)
    for f in r['fails']:
        print('  FAIL', f)
    torch.cuda.empty_cache()
