"""Training-loop fixture margins with the generator and discriminator precisions split:
prints, per fixture and (G, D) precision pair, the quantities closest to their bound.  Usage (GPU):
python tools/loop_margin.py [G:D ...]   e.g. x3:x3 x3:f32 f32:x3 f32:f32"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, 'explorable-super-resolution_old_amd'), REPO, os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)

import torch  # noqa: E402

from test_gpu_train_loop import TRAIN_CFGS, loop_margins  # noqa: E402

pairs = [a.split(':') for a in sys.argv[1:]] or [['x3', 'x3'], ['x3', 'f32'], ['f32', 'x3'], ['f32', 'f32']]
dev = torch.device('cuda:0')
for name in sorted(TRAIN_CFGS):
    for g, d in pairs:
        try:
            ok, rows = loop_margins(name, g, dev, d)
        except AssertionError as e:
            print('== %s  G=%s D=%s  trajectory left the fixture: %s' % (name, g, d, e))
            continue
        rows.sort(key=lambda r: -r[4])
        print('== %s  G=%s D=%s  flags %s  worst %.1f %%' % (name, g, d, 'ok' if ok else 'DIFFER', 100 * rows[0][4]))
        for kind, key, _, msg, _ in rows[:6]:
            print('   %-8s %-28s %s' % (kind, key, msg))
        sys.stdout.flush()
