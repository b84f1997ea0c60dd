"""GPU: the GUI's Z-optimisation objectives.
  * every objective case of tests/golden/zobj_cases.npz (the REFERENCE Z_optimizer's own run) with the stand-in model
    on the GPU — the objectives' device arithmetic (test_zobj_host.py runs the same on the CPU);
  * a selection of them on the HIP latent generator (RRDB + CEM, eval pre-pad, x3 and exact fp32) against the same
    objective loop with the CPU oracle as generator, in float64 and float32 (conftest.grad_parity on the Z update)."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import grad_parity

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))
from zobj_recipe import CASES, case_data  # noqa: E402
from test_zobj_host import FIX, check_case  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name', sorted(CASES))
def test_objective_matches_reference_gpu(gpu_device, name):
    """The first iteration of every case, and the whole run of every case that is not stiff (zobj_recipe.CASES: a
    1e4-weighted STD term makes later iterations amplify the GPU's other summation order)."""
    check_case(name, gpu_device, first=True)
    if not CASES[name].get('stiff'):
        check_case(name, gpu_device)


class _OracleNet(torch.nn.Module):
    def __init__(self, P, nb, dtype):
        super().__init__()
        from oracle import esr_oracle as O
        self.O, self.P, self.nb = O, {k: torch.as_tensor(v).to(dtype) for k, v in P.items()}, nb
        self.dummy = torch.nn.Parameter(torch.zeros(1, dtype=dtype))  # (Manage_Model_Grad_Requirements toggles it)
        self.dtype = dtype

    def forward(self, x):
        return self.O.sr_forward(x.to(self.dtype), self.P, self.nb, True, self.O.cem_design(4), pre_pad=True)


class _OracleModel:
    """SRRaGANModel's Z-optimisation surface over the CPU oracle (latent RRDB + CEM eval with pre-pad)."""

    def __init__(self, P, nb, lr, z, dtype):
        self.device = torch.device('cpu')
        self.num_latent_channels = 3
        self.netG = _OracleNet(P, nb, dtype)
        self.feed_data({'LR': lr, 'Z': z})
        with torch.no_grad():
            self.fake_H = self.netG(self.model_input)

    def feed_data(self, data, need_HR=True):
        lr, z = data['LR'], data['Z']
        B, _, h, w = lr.shape
        self.var_L, self.cur_Z = lr, z
        self.model_input = torch.cat([z.reshape(B, 48, h, w), lr], 1)

    def GetLatent(self):
        return self.cur_Z


def _opt(nb):
    return {'is_train': False, 'scale': 4, 'gpu_ids': [0], 'range': [0, 1],
            'network_G': {'which_model_G': 'RRDB_net', 'CEM_arch': 1, 'latent_input': 'all_layers',
                          'latent_input_domain': 'HR_downscaled', 'latent_channels': 'SVDinNormedOut_structure_tensor',
                          'norm_type': None, 'mode': 'CNA', 'nf': 64, 'nb': nb, 'in_nc': 3, 'out_nc': 3, 'gc': 32}}


def _data(data, dev):
    out = {}
    for k, v in data.items():
        if k == 'HR':
            out[k] = [torch.from_numpy(x).to(dev) for x in v] if isinstance(v, list) else torch.from_numpy(v).to(dev)
        else:
            out[k] = v
    return out


@pytest.mark.parametrize('name,precision', [('patchdict_noDC', 'x3'), ('patchdict_noDC', 'f32'), ('scribble', 'x3'),
                                            ('local_STD_nonInt_periodicity', 'x3'), ('local_Mag_increase', 'x3')])
def test_objective_on_hip_generator_vs_oracle(gpu_device, name, precision):
    from esr_amd import engine
    from esr_amd.SRRaGAN_model import SRRaGANModel
    from esr_amd.Z_optimization import Z_optimizer
    from oracle.recipe import seeded_params
    seed = int(FIX['%s:seed' % name])
    objective, B, data, img_mask, z_mask, z_range, lr, z, iters, lr0 = case_data(name, seed)
    iters = 3
    nb = 1
    torch.manual_seed(0)
    model = SRRaGANModel(_opt(nb), device=gpu_device)
    sd = model.netG.module.state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], seed + 5, w_scale=0.5)
    model.netG.module.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    engine.set_precision(model.netG, precision)
    lr_t, z_t = torch.from_numpy(lr), torch.from_numpy(z)
    gdata = dict(_data(data, gpu_device), LR=lr_t.to(gpu_device), Z=z_t.to(gpu_device))
    model.feed_data(gdata, need_HR=False)
    model.test()
    model.netG.eval()
    zo = Z_optimizer(objective, [4 * lr.shape[2], 4 * lr.shape[3]], model, z_range, iters, data=gdata,
                     initial_LR=lr0, image_mask=img_mask, Z_mask=z_mask, initial_Z=z_t.to(gpu_device), batch_size=B)
    z_gpu = zo.optimize().cpu().double()
    from oracle import esr_oracle as O
    P = O.strip_prefix(params)
    outs = []
    for dt in (torch.float64, torch.float32):
        om = _OracleModel(P, nb, lr_t.to(dt), z_t.to(dt), dt)
        cdata = dict(_data(data, 'cpu'), LR=lr_t.to(dt), Z=z_t.to(dt))
        zc = Z_optimizer(objective, [4 * lr.shape[2], 4 * lr.shape[3]], om, z_range, iters, data=cdata,
                         initial_LR=lr0, image_mask=img_mask, Z_mask=z_mask, initial_Z=z_t, batch_size=B)
        outs.append(zc.optimize().double())
    z0 = z_t.double()
    ok, msg = grad_parity(z_gpu - z0, outs[0] - z0, outs[1] - z0, floor=1e-4)
    print(name, precision, msg)
    assert ok, msg
