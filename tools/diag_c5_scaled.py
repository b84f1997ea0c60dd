"""Is the config-5 x3 dZ error set by the split-f16 precision of SMALL activations (lo parts below f16's normal range)?
The generator + CEM is linear in (activations, biases) jointly, so running it with every bias and the inputs (LR, Z)
multiplied by a power of two S gives S·output and the same input gradients — with every split activation S times
larger.  Prints tests/grid_parity.c5_z_gradients' lines for S = 1, 2^4, 2^8."""
import json
import os
import sys

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
for _p in (_R, os.path.join(_R, 'explorable-super-resolution_old_amd'), os.path.join(_R, 'tests')):
    sys.path.insert(0, _p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import grid_parity as GP  # noqa: E402


def run(S, precision='x3'):
    import esr_amd
    from esr_amd import CEMnet as C
    from esr_amd import engine
    from oracle.recipe import seeded_inputs, seeded_params
    d = np.load(os.path.join(_R, 'tests', 'golden', 'grid_c5_zgrad.npz'))
    cfg = json.loads(str(d['cfg']))
    B, h, K = cfg['B'], cfg['h'], cfg['proj']
    dev = torch.device('cuda', 0)
    net = esr_amd.RRDBNet(3, 3, 64, cfg['nb'], latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=d['kernel']).WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    params = seeded_params([(n, tuple(v.shape)) for n, v in sd.items()], cfg['seed'], w_scale=cfg['w_scale'])
    params = {n: (v * S if n.endswith('bias') and 'Filter' not in n else v) for n, v in params.items()}
    model.load_state_dict({n: torch.from_numpy(v) for n, v in params.items()}, strict=False)
    model = model.to(dev)
    model.eval()
    engine.set_precision(model, precision)
    for q in model.parameters():
        q.requires_grad = False
    lr, z = seeded_inputs(cfg['seed'] + 1, (B, 3, h, h), (B, 3, 4 * h, 4 * h), z_mode='pixel')
    R = np.random.default_rng(cfg['seed'] + 2).standard_normal((B, 3, 4 * h, 4 * h)).astype(np.float32)
    zt = torch.from_numpy(z * S).to(dev).requires_grad_(True)
    lt = torch.from_numpy(lr * S).to(dev).requires_grad_(True)
    out = model(torch.cat([zt.view(B, 48, h, h), lt], 1)) / S
    (out * torch.from_numpy(R).to(dev)).sum().backward()
    for i in cfg['images']:
        for name, v in (('dz', zt.grad[i] * S), ('dlr', lt.grad[i] * S), ('out', out.detach()[i])):
            mine = GP._proj(v.double().cpu().numpy(), cfg['seed'] + {'dz': 10, 'dlr': 11, 'out': 12}[name], i, K)
            p64, p32 = d['f64_%s_proj:%d' % (name, i)], d['f32_%s_proj:%d' % (name, i)]
            err, base, norm = np.linalg.norm(mine - p64), np.linalg.norm(p32 - p64), np.linalg.norm(p64)
            bound = 1e-4 * norm if name == 'out' else 5 * base + 1e-4 * norm
            print('S=%-6g %s image %d %-4s err %.3e bound %.3e (%.1f %%)' % (S, precision, i, name, err, bound,
                                                                          100 * err / bound), flush=True)
    del model, out, zt, lt
    torch.cuda.empty_cache()


for S in (1.0, 16.0, 256.0):
    run(S)
