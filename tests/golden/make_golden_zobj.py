"""Z-optimisation objective fixtures: the REFERENCE's Z_optimizer (codes/Z_optimization.py, read-only at
/root/reference) run here on the CPU over the stand-in model of tests/golden/zobj_recipe.py for every objective the
GUI builds (zobj_recipe.CASES).  Only the small .npz it writes is committed.

    python tests/golden/make_golden_zobj.py [case ...]
    python tests/golden/make_golden_zobj.py auto_hist     (what auto_set_hist_temperature raises -> zobj_auto_hist.json)

In-memory shims (nothing is written under /root/reference; no reference bytecode is loaded or written), on top of
make_golden.install_shims():
  1. torch.device('cuda') targets: Tensor.to / Module.to map a CUDA device to the CPU (the reference moves everything
     to torch.device('cuda'), Z_optimization.py:29,345).
  2. skimage is absent: `skimage.color.rgb2hsv / hsv2rgb` (used by the scribble objective only,
     Z_optimization.py:388-391) are restated from scikit-image's published algorithm (skimage/color/colorconv.py:
     V = max, S = (max − min)/max, H from the max channel's sector; the inverse by the six-sector choose).  The
     scribble case is therefore pinned to this restatement of the colour conversion.
  3. `1 - mask` of a comparison mask (Z_optimization.py:393) — the reference's PyTorch returned uint8 from comparisons
     and their sums; this one returns bool, whose subtraction raises: a bool operand of Tensor.__rsub__ is taken as
     uint8, the reference's semantics.
  4. `mask ^ 1` of a comparison mask (Desired_Im_2_Bins, Z_optimization.py:120): with the reference's uint8 masks a
     logical NOT that is then used as a mask index; on a bool tensor this PyTorch promotes the result to int64, which
     would index with 0/1 positions instead.  A bool operand of Tensor.__xor__ with an int is taken as uint8.
  5. torch.normal (the 'random…limited' objectives' initial perturbation, Z_optimization.py:285) draws from a seeded
     NumPy stream that the GPU test replays.
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
sys.pycache_prefix = '/tmp/esr_golden_pycache'

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402
from zobj_recipe import CASES, FIRST_ITERS, StandInModel, case_data  # noqa: E402


def _rgb2hsv(rgb):
    arr = np.asarray(rgb, dtype=np.float64)
    v = arr.max(-1)
    delta = arr.max(-1) - arr.min(-1)
    with np.errstate(invalid='ignore', divide='ignore'):
        s = delta / v
        s[delta == 0.0] = 0.0
        h = np.zeros_like(v)
        for c, (a, b, off) in enumerate(((1, 2, 0.0), (2, 0, 2.0), (0, 1, 4.0))):
            idx = arr[..., c] == v
            h[idx] = off + (arr[idx, a] - arr[idx, b]) / delta[idx]
        h = (h / 6.0) % 1.0
        h[delta == 0.0] = 0.0
    return np.stack([h, s, v], -1)


def _hsv2rgb(hsv):
    arr = np.asarray(hsv, dtype=np.float64)
    hi = np.floor(arr[..., 0] * 6)
    f = arr[..., 0] * 6 - hi
    p = arr[..., 2] * (1 - arr[..., 1])
    q = arr[..., 2] * (1 - f * arr[..., 1])
    t = arr[..., 2] * (1 - (1 - f) * arr[..., 1])
    v = arr[..., 2]
    hi = np.stack([hi, hi, hi], -1).astype(np.uint8) % 6
    return np.choose(hi, np.stack([np.stack((v, t, p), -1), np.stack((q, v, p), -1), np.stack((p, v, t), -1),
                                   np.stack((p, q, v), -1), np.stack((t, p, v), -1), np.stack((v, p, q), -1)]))


NOISE = {}


def install_zobj_shims():
    make_golden.install_shims()
    sk = types.ModuleType('skimage')
    col = types.ModuleType('skimage.color')
    col.rgb2hsv, col.hsv2rgb = _rgb2hsv, _hsv2rgb
    sk.color = col
    sys.modules['skimage'], sys.modules['skimage.color'] = sk, col

    def cpu(d):
        return 'cpu' if (isinstance(d, torch.device) and d.type == 'cuda') or (isinstance(d, str) and
                                                                             d.startswith('cuda')) else d
    t_to, m_to = torch.Tensor.to, torch.nn.Module.to
    torch.Tensor.to = lambda self, *a, **k: t_to(self, *[cpu(x) for x in a], **{n: cpu(v) for n, v in k.items()})
    torch.nn.Module.to = lambda self, *a, **k: m_to(self, *[cpu(x) for x in a], **{n: cpu(v) for n, v in k.items()})

    rsub = torch.Tensor.__rsub__
    torch.Tensor.__rsub__ = lambda self, other: rsub(self.to(torch.uint8) if self.dtype == torch.bool else self, other)

    xor = torch.Tensor.__xor__
    torch.Tensor.__xor__ = lambda self, other: xor(self.to(torch.uint8), other) \
        if self.dtype == torch.bool and isinstance(other, int) else xor(self, other)

    def normal(mean, std, *a, **k):
        rng = NOISE['rng']
        return mean + std * torch.from_numpy(rng.standard_normal(tuple(mean.shape)).astype(np.float32))
    torch.normal = normal


def run_case(Zo, name, seed, iters_override=None):
    objective, B, data, img_mask, z_mask, z_range, lr, z, iters, lr0 = case_data(name, seed)
    iters = iters_override or iters
    torch.manual_seed(0)
    NOISE['rng'] = np.random.default_rng(seed + 7)
    model = StandInModel(torch.from_numpy(lr), torch.from_numpy(z), seed + 3, 'cpu')
    tdata = {'LR': torch.from_numpy(lr)}
    for k, v in data.items():
        if k == 'HR':
            tdata[k] = [torch.from_numpy(x) for x in v] if isinstance(v, list) else torch.from_numpy(v)
        else:
            tdata[k] = v
    zo = Zo.Z_optimizer(objective=objective, Z_size=[4 * lr.shape[2], 4 * lr.shape[3]], model=model, Z_range=z_range,
                        max_iters=iters, data=tdata, initial_LR=lr0, image_mask=img_mask, Z_mask=z_mask,
                        initial_Z=torch.from_numpy(z), batch_size=B)
    z_out = zo.optimize()
    out = {'loss_values': np.array(zo.loss_values, dtype=np.float64), 'z_out': z_out.detach().numpy(),
           'latest': np.array(zo.latest_Z_loss_values, dtype=np.float64),
           'fake_H': model.fake_H.detach().numpy()}
    print('%-36s %s: loss %s' % (name, objective, ['%.6e' % v for v in zo.loss_values]), flush=True)
    return out


def auto_hist_temperature(Zo):
    """The reference's auto_set_hist_temperature (Z_optimization.py:476-499) on a 'hist' case with the GUI's data
    layout (data['HR'] a list of desired images, GUI.py:1549): what it raises, recorded in zobj_auto_hist.json."""
    out = {}
    for name in ('hist_localSTD', 'patchhist_noDC_localSTD'):
        objective, B, data, img_mask, z_mask, z_range, lr, z, iters, lr0 = case_data(name, 1234)
        torch.manual_seed(0)
        model = StandInModel(torch.from_numpy(lr), torch.from_numpy(z), 1237, 'cpu')
        tdata = {'LR': torch.from_numpy(lr), 'HR': [torch.from_numpy(x) for x in data['HR']],
                 'Desired_Im_Mask': data['Desired_Im_Mask']}
        try:
            Zo.Z_optimizer(objective=objective, Z_size=[4 * lr.shape[2], 4 * lr.shape[3]], model=model,
                           Z_range=z_range, max_iters=iters, data=tdata, initial_LR=lr0, image_mask=img_mask,
                           Z_mask=z_mask, initial_Z=torch.from_numpy(z), batch_size=B, auto_set_hist_temperature=True)
            out[name] = {'raises': None}
        except Exception as e:  # noqa: BLE001
            out[name] = {'raises': type(e).__name__, 'message': str(e)}
        print(name, out[name], flush=True)
    with open(os.path.join(HERE, 'zobj_auto_hist.json'), 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)


def main():
    install_zobj_shims()
    import Z_optimization as Zo
    if sys.argv[1:] == ['auto_hist']:
        auto_hist_temperature(Zo)
        return
    torch.set_num_threads(8)
    names = sys.argv[1:] or list(CASES)
    path = os.path.join(HERE, 'zobj_cases.npz')
    d = dict(np.load(path)) if os.path.exists(path) and sys.argv[1:] else {}
    for i, name in enumerate(sorted(CASES)):
        if name not in names:
            continue
        seed = 900 + 10 * i
        for k, v in run_case(Zo, name, seed).items():
            d['%s:%s' % (name, k)] = v
        # the first iteration alone ('random…limited': two — the reference overwrites loss_values[0] with [1])
        for k, v in run_case(Zo, name, seed, iters_override=FIRST_ITERS(name)).items():
            d['%s:%s1' % (name, k)] = v
        d['%s:seed' % name] = np.int64(seed)
    d['cases'] = np.str_(json.dumps(sorted(CASES)))
    np.savez_compressed(path, **d)


if __name__ == '__main__':
    main()
