"""Stand-in SR model and seeded data for the Z-optimisation objective fixtures (tests/golden/make_golden_zobj.py runs the
REFERENCE Z_optimizer on them on the CPU; tests/test_gpu_zobj.py runs esr_amd's Z_optimizer on them on the GPU).

The stand-in keeps only what Z_optimizer touches on its model (Z_optimization.py:329-655: netG, feed_data,
model_input, fake_H, GetLatent, num_latent_channels): a small smooth generator fake_H = sigmoid(2·(up4(LR) − ½) +
conv3x3(Z)), so the objectives — the part these fixtures pin — are exercised on the same images on both sides.  The
RRDB/CEM generator under the objectives is pinned separately (zgrad_* / grid_c5_zgrad fixtures, test_gpu_zopt.py).

TEST INFRASTRUCTURE ONLY (no reference code)."""
import numpy as np
import torch
import torch.nn.functional as F


class StandInG(torch.nn.Module):
    def __init__(self, seed):
        super().__init__()
        rng = np.random.default_rng(seed)
        self.weight = torch.nn.Parameter(torch.from_numpy((0.4 * rng.standard_normal((3, 3, 3, 3))).astype(np.float32)))
        self.bias = torch.nn.Parameter(torch.from_numpy((0.1 * rng.standard_normal(3)).astype(np.float32)))

    def forward(self, inp):
        lr, z = inp
        up = F.interpolate(lr, scale_factor=4, mode='nearest')
        return torch.sigmoid(2 * (up - 0.5) + F.conv2d(z, self.weight, self.bias, padding=1))


class StandInModel:
    """What Z_optimizer reads and calls on SRRaGANModel."""

    def __init__(self, lr, z, seed, device):
        self.device = torch.device(device)
        self.num_latent_channels = 3
        self.Z_size_factor = 4
        self.netG = StandInG(seed).to(self.device)
        self.var_L = lr.to(self.device)
        self.cur_Z = z.to(self.device)
        self.model_input = (self.var_L, self.cur_Z)
        with torch.no_grad():
            self.fake_H = self.netG(self.model_input)

    def feed_data(self, data, need_HR=True):
        self.var_L = data['LR']
        self.cur_Z = data['Z']
        self.model_input = (self.var_L, self.cur_Z)

    def GetLatent(self):
        return self.cur_Z


H = W = 48  # HR size (LR 12 x 12)


def _blob(h, w, seed, cy, cx, ry, rx):
    """A ragged elliptical mask (float64 0/1) with a few seeded holes on its rim."""
    yy, xx = np.mgrid[0:h, 0:w]
    m = (((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0).astype(np.float64)
    rng = np.random.default_rng(seed)
    edge = np.argwhere((((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 > 0.8) & (m > 0))
    for i in rng.choice(len(edge), size=len(edge) // 5, replace=False):
        m[tuple(edge[i])] = 0.0
    return m


def case_data(name, seed):
    """(objective, batch, data dict of NumPy arrays / lists, image_mask, Z_mask, Z_range, lr, iters) of one case."""
    rng = np.random.default_rng(seed)
    spec = CASES[name]
    B = spec.get('batch', 1)
    lr = rng.random((B, 3, H // 4, W // 4)).astype(np.float32)
    z = (0.6 * rng.random((B, 3, H, W)) - 0.3).astype(np.float32)
    img_mask = _blob(H, W, seed + 1, 23.5, 25.0, 17.0, 19.0)
    z_mask = np.clip(img_mask + np.roll(img_mask, 1, 0) + np.roll(img_mask, -1, 1), 0, 1)
    data = {}
    if spec.get('hist'):
        dh, dw = 40, 44
        desired = rng.random((1, 3, dh, dw)).astype(np.float32)
        desired = (0.5 * desired + 0.5 * np.round(desired * 4) / 4).astype(np.float32)  # a few dominant levels
        data['HR'] = [desired]
        data['Desired_Im_Mask'] = [_blob(dh, dw, seed + 2, 20.0, 22.0, 17.0, 19.0)]
    if 'STD_increment' in spec:
        data['STD_increment'] = spec['STD_increment']
    if 'points' in spec:
        data['periodicity_points'] = [np.array(p) for p in spec['points']]  # ints: integer shifts
    if spec.get('scribble'):
        sm = np.zeros((H, W), dtype=np.int64)
        sm[8:20, 10:30] = 1   # L1 to the scribbled image
        sm[22:30, 8:22] = 2   # brighten
        sm[22:30, 26:40] = 3  # darken
        sm[32:44, 12:36] = 5  # local TV region
        sm[34:38, 38:46] = 7  # a second TV region
        data['scribble_mask'] = sm
        data['brightness_factor'] = 0.3
        data['HR'] = rng.random((1, 3, H, W)).astype(np.float32)
    if 'rmse_weight' in spec:
        data['rmse_weight'] = spec['rmse_weight']
    return (spec['objective'], B, data, img_mask if spec.get('masks', True) else None,
            z_mask if spec.get('masks', True) else None, spec.get('Z_range', 1.0), lr, z, spec.get('iters', 4),
            spec.get('lr', 0.05))


# stiff=True: a 1e4-weighted STD-preservation term ('localSTD', also inside 'no_localSTD') makes every Adam step
# overshoot, so after the first iteration the trajectory amplifies rounding differences (the loss jumps by 100x from
# one iteration to the next in the reference itself); tests compare those cases' later iterations only where the
# arithmetic order matches the reference's (the CPU) and their first iteration everywhere.
# The GUI's objective strings with its shipped switches (GUI.py:37-49, 1505-1517: LOCAL_STD_4_OPT, NO_DC_IN_PATCH_
# HISTOGRAM, DICTIONARY_REPLACES_HISTOGRAM, AUTO_CYCLE_LENGTH_4_PERIODICITY; 'special behaviour' -> Mag, Plus,
# no_localSTD), plus the plain forms
CASES = {
    'local_STD_increase': dict(objective='local_STD_increase', STD_increment=0.02),
    'local_STD_decrease': dict(objective='local_STD_decrease', STD_increment=0.02, batch=2),
    'local_max_STD': dict(objective='local_max_STD'),
    'STD_increase_masked': dict(objective='STD_increase', STD_increment=None),
    'local_STD_TV': dict(objective='local_STD_TV'),
    'TV_masked': dict(objective='TV'),
    'dict_noDC': dict(objective='dict_noDC', hist=True),
    'patchdict_noDC': dict(objective='patchdict_noDC', hist=True),
    'patchdict_noDC_no_localSTD': dict(objective='patchdict_noDC_no_localSTD', hist=True, stiff=True),
    'hist_localSTD': dict(objective='hist_localSTD', hist=True, stiff=True),
    'patchhist_noDC_localSTD': dict(objective='patchhist_noDC_localSTD', hist=True, stiff=True),
    'local_STD_nonInt_periodicity': dict(objective='local_STD_nonInt_periodicity',
                                         points=[[3.3, 1.2], [-0.8, 4.1]]),
    'local_STD_nonInt_periodicity_1D': dict(objective='local_STD_nonInt_periodicity_1D', points=[[2.6, 2.6]]),
    'local_STD_nonInt_periodicityPlus': dict(objective='local_STD_nonInt_periodicityPlus', STD_increment=0.01,
                                             points=[[3.5, 0.0], [0.0, 3.0]]),
    'periodicity_int': dict(objective='periodicity', points=[[4, 0], [0, 3]]),
    'scribble': dict(objective='scribble', scribble=True),
    'local_Mag_increase': dict(objective='local_Mag_increase', STD_increment=0.05),
    'local_Mag_decrease': dict(objective='local_Mag_decrease', STD_increment=0.05),
    'random_l1': dict(objective='random_l1', batch=3, lr=0.1),
    'random_l1_limited': dict(objective='random_l1_limited', batch=2, rmse_weight=0.5, lr=0.1),
}


def FIRST_ITERS(name):
    """Iterations of a case's short run (the first iteration; two for 'random…limited', whose reference loop reads
    loss_values[1], Z_optimization.py:644)."""
    return 2 if 'limited' in CASES[name]['objective'] else 1
