import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, '.'); sys.path.insert(0, 'explorable-super-resolution_old_amd')
import numpy as np, torch
import esr_amd
from oracle import esr_oracle as O
from oracle.recipe import seeded_params, seeded_inputs
dev = torch.device('cuda', 0)
for (h, w, latent) in [(38, 38, True), (38, 38, False), (32, 32, False), (40, 40, False)]:
    net = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    params = seeded_params([(k, tuple(v.shape)) for k, v in net.state_dict().items()], 5, w_scale=0.5)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    net = net.to(dev).train(True)
    lr, z = seeded_inputs(6, (1, 3, h, w), (1, 3, 4 * h, 4 * w) if latent else None, z_mode='pixel')
    x = torch.from_numpy(lr)
    if latent:
        x = torch.cat([torch.from_numpy(z).view(1, 48, h, w), x], 1)
    R = torch.from_numpy(np.random.default_rng(7).standard_normal((1, 3, 4 * h, 4 * w)).astype(np.float32))
    xg = x.to(dev).requires_grad_(True)
    out = net(xg); (out * R.to(dev)).sum().backward()
    P = {k: torch.as_tensor(v).double().requires_grad_(True) for k, v in params.items()}
    xr = x.double().requires_grad_(True)
    ref = O.rrdbnet_forward(xr, P, 1, latent); (ref * R.double()).sum().backward()
    def rel(a, b): return float((a.double().cpu() - b).abs().max() / b.abs().max())
    worst = max(((rel(p.grad, P[n].grad), n) for n, p in net.named_parameters()))
    print(h, w, latent, 'fwd %.2e' % rel(out.detach(), ref.detach()), 'worst param grad %.2e %s' % worst,
          'dx %.2e' % rel(xg.grad, xr.grad))
