"""Is the training step deterministic?  Runs the training-loop fixture's configuration twice in one process (and
reports a third run's first micro-step) and compares per-micro-step digests of every G / D parameter and D buffer
bitwise.  Usage (GPU): python tools/loop_determinism.py [G:D] [fixture]"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, 'explorable-super-resolution_old_amd'), REPO, os.path.join(REPO, 'tests'),
          os.path.join(REPO, 'tests', 'golden')):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_train_loop as T  # noqa: E402
from train_recipe import step_data  # noqa: E402

g, d = (sys.argv[1] if len(sys.argv) > 1 else 'x3:f32').split(':')
name = sys.argv[2] if len(sys.argv) > 2 else 'adaptive_rel'
dev = torch.device('cuda:0')
cfg = json.loads(str(np.load(os.path.join(REPO, 'tests', 'golden', 'train_%s.npz' % name))['cfg']))


def digest(t):
    return hashlib.sha1(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:12]


def run():
    # T._run_port with a per-micro-step digest hook
    from esr_amd import dconv
    prev = dconv.PRECISION
    orig = T.step_data
    rows = []
    model_box = {}

    def hooked(c, k):
        m = model_box.get('m')
        if m is not None and k > 0:
            dg = {'Dgrad.' + n: p.grad.detach().clone() for n, p in m.netD.named_parameters() if p.grad is not None}
            rows.append((k - 1, {n: digest(v) for n, v in list(m.netG.state_dict().items()) +
                                 [('D.' + n, v) for n, v in m.netD.state_dict().items()]}, dg))
        return orig(c, k)
    T.step_data = hooked
    from esr_amd.SRRaGAN_model import SRRaGANModel
    init = SRRaGANModel.__init__

    def grab(self, *a, **kw):
        init(self, *a, **kw)
        model_box['m'] = self
    SRRaGANModel.__init__ = grab
    try:
        model, _, _, flags = T._run_port(cfg, g, dev, d)
    finally:
        T.step_data = orig
        SRRaGANModel.__init__ = init
        dconv.set_precision(prev)
    rows.append((cfg['steps'] - 1, {n: digest(v) for n, v in list(model.netG.state_dict().items()) +
                                    [('D.' + n, v) for n, v in model.netD.state_dict().items()]}, {}))
    return rows, {k: list(v) for k, v in model.log_dict.items()}


a, la = run()
b, lb = run()
c, lc = run()
print('G=%s D=%s %s: %d micro-steps; run 2 == run 3: %s' % (
    g, d, name, len(a), all(x[1] == y[1] for x, y in zip(b, c)) and lb == lc))
for (k, da, ga), (_, db, gb) in zip(a, b):
    diff = [n for n in da if da[n] != db[n]]
    gd = [(n, float((ga[n] - gb[n]).abs().max() / ga[n].abs().max().clamp_min(1e-30))) for n in ga
          if not torch.equal(ga[n], gb[n])]
    print('after micro-step %d: %d of %d tensors differ %s; D grads differing (max rel): %s' % (
        k, len(diff), len(da), diff[:6], gd[:8]))
    if diff:
        break
print('logs equal:', la == lb)
