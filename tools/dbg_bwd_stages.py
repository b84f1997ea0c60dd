import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, '.'); sys.path.insert(0, 'explorable-super-resolution_old_amd')
import numpy as np, torch
import torch.nn.functional as F
import esr_amd
from oracle import esr_oracle as O
from oracle.recipe import seeded_params, seeded_inputs
dev = torch.device('cuda', 0)
L = 0.2
for (h, w) in [(38, 38), (40, 40)]:
    net = esr_amd.RRDBNet(3, 3, 64, 1, num_latent_channels=0)
    params = seeded_params([(k, tuple(v.shape)) for k, v in net.state_dict().items()], 5, w_scale=0.5)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    net = net.to(dev).train(True)
    lr, _ = seeded_inputs(6, (1, 3, h, w), None)
    R = torch.from_numpy(np.random.default_rng(7).standard_normal((1, 3, 4 * h, 4 * w)).astype(np.float32))
    out = net(torch.from_numpy(lr).to(dev)); (out * R.to(dev)).sum().backward()
    ws = net._esr_cache['train_ws'][1]
    P = {k: torch.as_tensor(v).double() for k, v in params.items()}
    x = torch.from_numpy(lr).double().requires_grad_(True)
    cv = lambda t, k: F.conv2d(t, P[k + '.weight'], P[k + '.bias'], padding=1)
    fea = cv(x, 'model.0'); fea.retain_grad()
    t = O._rrdb(fea, P, 'model.1.sub.0', None); t.retain_grad()
    u0 = fea + cv(t, 'model.1.sub.1'); u0.retain_grad()
    a1 = cv(F.interpolate(u0, scale_factor=2, mode='nearest'), 'model.2.1'); a1.retain_grad()
    up1 = F.leaky_relu(a1, L)
    n1 = F.interpolate(up1, scale_factor=2, mode='nearest'); n1.retain_grad()
    a2 = cv(n1, 'model.3.1'); a2.retain_grad()
    up2 = F.leaky_relu(a2, L)
    a3 = cv(up2, 'model.4'); a3.retain_grad()
    h0 = F.leaky_relu(a3, L)
    o = cv(h0, 'model.6')
    print(h, w, 'fwd %.2e' % float((out.detach().cpu().double() - o).abs().max() / o.abs().max()))
    (o * R.double()).sum().backward()
    def cmp(name, buf, ref, c0=0):
        g = buf[:, 1:-1, 1:-1, c0:c0 + ref.shape[1]].permute(0, 3, 1, 2).cpu().double()
        e = (g - ref.grad).abs()
        print('  %-22s rel %.2e' % (name, float(e.max() / ref.grad.abs().max())), 'bad px', int((e.amax(1) > 1e-4 * ref.grad.abs().max()).sum()))
    dA, dB = ws.dHR
    cmp('dB = d a2 (pre-act)', dB, a2)
    cmp('dA = d n1 (4H)', dA, n1)
    cmp('dU1 = d a1', ws.dU1, a1)
    cmp('dU0 = d u0', ws.dU0, u0)
    cmp('GA = d fea', ws.GA, fea)
