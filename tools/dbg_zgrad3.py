import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, '.'); sys.path.insert(0, 'explorable-super-resolution_old_amd')
import numpy as np, torch
import torch.nn.functional as F
from conftest import golden, fixture_params
import esr_amd
from esr_amd import CEMnet as C
from oracle import esr_oracle as O
dev = torch.device('cuda', 0)
for name in ['zgrad_eval', 'zgrad_eval_learned']:
    d = golden(name); _, params = fixture_params(d)
    kern = d['kernel'] if 'kernel' in d.files else None
    net = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    cem = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=kern)
    model = cem.WrapArchitecture_PyTorch(net)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    model = model.to(dev).eval()
    for p in model.parameters(): p.requires_grad = False
    z = torch.from_numpy(d['z']).to(dev).requires_grad_(True); lr = torch.from_numpy(d['lr']).to(dev).requires_grad_(True)
    B, _, h, w = lr.shape
    R = torch.from_numpy(d['R'])
    out = model(torch.cat([z.view(B, 48, h, w), lr], 1)); (out * R.to(dev)).sum().backward()
    ws = net._esr_cache['train_ws'][1]
    dgen = ws.dgen_p[:, 1:-1, 1:-1, :3].permute(0, 3, 1, 2).cpu().double()
    dfirst = ws.dFirst[:, 1:-1, 1:-1].permute(0, 3, 1, 2).cpu().double()
    dzl = ws.dZl[:, 1:-1, 1:-1, :3].permute(0, 3, 1, 2).cpu().double()
    # oracle in float64 with the intermediate gradients
    design = O.cem_design(4, kern)
    P = {k: torch.as_tensor(v).double() for k, v in O.strip_prefix(params).items()}
    mL, mH = design['margins_LR'], design['margins_HR']
    zr = torch.from_numpy(d['z']).double(); lrr = torch.from_numpy(d['lr']).double()
    zp = F.pad(zr, (mH,) * 4, mode='replicate').requires_grad_(True)
    lp = F.pad(lrr, (mL,) * 4, mode='replicate').requires_grad_(True)
    H, W = h + 2 * mL, w + 2 * mL
    zlr = O.bilinear_down4(zp); zlr.retain_grad()
    # re-run the generator with z_lr as an explicit leaf to get its gradient
    x = torch.cat([zp.reshape(B, 48, H, W), lp], 1)
    gen = O.rrdbnet_forward(x, P, 1, True); gen.retain_grad()
    ds, inv = design['ds_kernel'], design['inv_hTh']
    o = O.cem_upscale(O.cem_inv(lp, inv), ds) + gen - O.cem_upscale(O.cem_inv(O.cem_downscale(gen, ds), inv), ds)
    o = o[:, :, mH:-mH, mH:-mH]
    (o * R.double()).sum().backward()
    def rel(a, b): return float((a - b).abs().max() / b.abs().max())
    print(name, 'dgen rel %.2e' % rel(dgen, gen.grad))
    e = (dgen - gen.grad).abs().amax(dim=(0, 1)); print('  dgen err col prof', (e.amax(0) / gen.grad.abs().max() * 1e6).round().int().tolist()[:60])
    print('  dgen err row prof', (e.amax(1) / gen.grad.abs().max() * 1e6).round().int().tolist()[:60])
