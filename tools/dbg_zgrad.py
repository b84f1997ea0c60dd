import sys, os
sys.path.insert(0, 'tests'); sys.path.insert(0, '.'); sys.path.insert(0, 'explorable-super-resolution_old_amd')
import numpy as np, torch
from conftest import golden, fixture_params, normwise_rel
import esr_amd
from esr_amd import CEMnet as C
dev = torch.device('cuda', 0)
for name in ['zgrad_eval', 'zgrad_eval_learned']:
    d = golden(name); _, params = fixture_params(d)
    net = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    cem = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=d['kernel'] if 'kernel' in d.files else None)
    model = cem.WrapArchitecture_PyTorch(net)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    model = model.to(dev).eval()
    for p in model.parameters(): p.requires_grad = False
    z = torch.from_numpy(d['z']).to(dev).requires_grad_(True)
    lr = torch.from_numpy(d['lr']).to(dev).requires_grad_(True)
    B, _, h, w = lr.shape
    out = model(torch.cat([z.view(B, 48, h, w), lr], 1))
    (out * torch.from_numpy(d['R']).to(dev)).sum().backward()
    for nm, g, ref in (('dz', z.grad.cpu().numpy(), d['dz']), ('dlr', lr.grad.cpu().numpy(), d['dlr'])):
        e = np.abs(g - ref)
        print(name, nm, 'rel %.2e' % (e.max() / np.abs(ref).max()), 'argmax', np.unravel_index(e.argmax(), e.shape), 'shape', e.shape)
        em = e.max(axis=(0, 1))
        print('  row max err', np.round(em.max(axis=1) / np.abs(ref).max() * 1e6).astype(int).tolist())
        print('  col max err', np.round(em.max(axis=0) / np.abs(ref).max() * 1e6).astype(int).tolist())
    print('margins', cem.invalidity_margins_LR, cem.invalidity_margins_HR, 'ds', cem.ds_kernel.shape, 'inv', cem.inv_hTh.shape)
