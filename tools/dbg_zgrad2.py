import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, '.'); sys.path.insert(0, 'explorable-super-resolution_old_amd')
import numpy as np, torch
from conftest import normwise_rel
import esr_amd
from esr_amd import CEMnet as C
from oracle import esr_oracle as O
from oracle.recipe import seeded_params, seeded_inputs
dev = torch.device('cuda', 0)
for (h, w, mode) in [(38, 38, 'bare'), (38, 38, 'train'), (32, 32, 'bare'), (24, 38, 'bare'), (38, 24, 'bare'), (40, 40, 'bare')]:
    net = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net) if mode != 'bare' else net
    params = seeded_params([(k, tuple(v.shape)) for k, v in model.state_dict().items()], 5, w_scale=0.5)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    model = model.to(dev).train(True)
    for p in model.parameters(): p.requires_grad = False
    lr, z = seeded_inputs(6, (1, 3, h, w), (1, 3, 4 * h, 4 * w), z_mode='pixel')
    R = torch.from_numpy(np.random.default_rng(7).standard_normal((1, 3, 4 * h, 4 * w)).astype(np.float32))
    zt = torch.from_numpy(z).to(dev).requires_grad_(True); lt = torch.from_numpy(lr).to(dev).requires_grad_(True)
    out = model(torch.cat([zt.view(1, 48, h, w), lt], 1)); (out * R.to(dev)).sum().backward()
    zr = torch.from_numpy(z).double().requires_grad_(True); lrr = torch.from_numpy(lr).double().requires_grad_(True)
    P = {k: torch.as_tensor(v).double() for k, v in O.strip_prefix(params).items()}
    ref = O.sr_forward(torch.cat([zr.view(1, 48, h, w), lrr], 1), P, 1, True, O.cem_design(4) if mode != 'bare' else None, pre_pad=False)
    (ref * R.double()).sum().backward()
    for nm, g, r in (('dz', zt.grad, zr.grad), ('dlr', lt.grad, lrr.grad)):
        e = (g.cpu().double() - r).abs(); s = r.abs().max()
        print(h, w, mode, nm, 'rel %.2e' % (e.max() / s), 'col prof', (e.amax(dim=(0, 1, 2)) / s * 1e6).round().int().tolist()[:12], 'row prof', (e.amax(dim=(0, 1, 3)) / s * 1e6).round().int().tolist()[:40])
