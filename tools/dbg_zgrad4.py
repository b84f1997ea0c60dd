import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, '.'); sys.path.insert(0, 'explorable-super-resolution_old_amd')
import numpy as np, torch
import torch.nn.functional as F
import esr_amd
from oracle import esr_oracle as O
from oracle.recipe import seeded_params, seeded_inputs
dev = torch.device('cuda', 0)


def fwd_leaf(lr, z_lr, z_hr, P, nb=1):
    x = torch.cat([z_lr, lr], 1)
    fea = O._conv(x, P, 'model.0', act=False)
    out = torch.cat([z_lr, fea], 1)
    for k in range(nb):
        if k > 0:
            out = torch.cat([z_lr, out], 1)
        out = O._rrdb(out, P, 'model.1.sub.%d' % k, z_lr)
    out = torch.cat([z_lr, out], 1)
    out = fea + O._conv(out, P, 'model.1.sub.%d' % nb, act=False)
    for key in ('model.2.1', 'model.3.1'):
        out = O._conv(F.interpolate(out, scale_factor=2, mode='nearest'), P, key, act=True)
    out = torch.cat([z_hr, out], 1)
    out = O._conv(out, P, 'model.4', act=True)
    out = torch.cat([z_hr, out], 1)
    return O._conv(out, P, 'model.6', act=False)


for (h, w) in [(38, 38), (32, 32), (40, 40)]:
    net = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    params = seeded_params([(k, tuple(v.shape)) for k, v in net.state_dict().items()], 5, w_scale=0.5)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    net = net.to(dev).train(True)
    lr, z = seeded_inputs(6, (1, 3, h, w), (1, 3, 4 * h, 4 * w), z_mode='pixel')
    R = torch.from_numpy(np.random.default_rng(7).standard_normal((1, 3, 4 * h, 4 * w)).astype(np.float32))
    zt = torch.from_numpy(z).to(dev).requires_grad_(True); lt = torch.from_numpy(lr).to(dev).requires_grad_(True)
    out = net(torch.cat([zt.view(1, 48, h, w), lt], 1)); (out * R.to(dev)).sum().backward()
    ws = net._esr_cache['train_ws'][1]
    P = {k: torch.as_tensor(v).double().requires_grad_(True) for k, v in params.items()}
    zh = torch.from_numpy(z).double().requires_grad_(True)
    zl = O.bilinear_down4(zh).detach().requires_grad_(True)
    lrr = torch.from_numpy(lr).double().requires_grad_(True)
    ref = fwd_leaf(lrr, zl, zh, P); (ref * R.double()).sum().backward()
    def rel(a, b): return float((a.double().cpu() - b).abs().max() / b.abs().max())
    print(h, w, 'fwd %.2e' % rel(out.detach(), ref.detach()))
    dzl = ws.dZl[:, 1:-1, 1:-1, :3].permute(0, 3, 1, 2)
    dfirst_z = ws.dFirst[:, 1:-1, 1:-1, :3].permute(0, 3, 1, 2)
    dfirst_l = ws.dFirst[:, 1:-1, 1:-1, 8:11].permute(0, 3, 1, 2)
    print('  dZ_LR total %.2e' % rel(dzl, zl.grad), ' dLR %.2e' % rel(dfirst_l, lrr.grad))
    e = (dzl.double().cpu() - zl.grad).abs()[0, 0]
    bad = (e > 1e-4 * zl.grad.abs().max()).nonzero()
    print('  bad LR px', bad.shape[0], bad[:12].tolist())
