"""Training and Z-optimisation parity at the PRODUCTION grids: the shape-dependent launch choices
(x3 weight-gradient split-K, per-RRDB gradient scales, discriminator tile / split-K modes, the halo-tile forward) run
exactly as in bench_train.py / bench_zopt.py.

* Config 3: SRRaGANModel.optimize_parameters, B=16 × 96² LR, RRDB-23, latent, CEM train mode (D at the unpadded HR
  size), WGAN-GP — two micro-steps (a D step, then a D + G step) against the REFERENCE's own optimize_parameters run
  on the same seeded weights and batches in float64 and float32 (tests/golden/make_golden_train.py c3).  Every G and
  D parameter gradient of the second step is compared through K seeded random projections (the fixture cannot hold
  16.7 M float64 gradients): relative L2 distance to the float64 run within 5× the reference's own float32 distance
  plus a floor of 1e-4 (conftest.grad_parity's yardstick); the logged D outputs / losses / gradient penalty and the D
  BatchNorm buffers as in test_gpu_train_loop.py."""
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))
from train_recipe import grad_projections  # noqa: E402

from test_gpu_train_loop import D_DIFFERENCES, _close, _run_port  # noqa: E402

pytestmark = pytest.mark.gpu

FACTOR, FLOOR = 5.0, 1e-4


@pytest.mark.parametrize('precision', ['x3', 'f32'])
def test_c3_training_step_at_production_grid(gpu_device, precision):
    path = os.path.join(HERE, 'golden', 'grid_c3_train.npz')
    d = np.load(path)
    cfg = json.loads(str(d['cfg']))
    from esr_amd import dconv
    prev = dconv.PRECISION
    try:
        model, _, _, flags = _run_port(cfg, precision, gpu_device)
    finally:
        dconv.set_precision(prev)
    assert flags == list(d['f64_generator_step']) == list(d['f32_generator_step']) == [False, True]
    fails, worst = [], 0.0
    for net, tag in ((model.netG, 'G'), (model.netD, 'D')):
        errs = []
        for i, (k, p) in enumerate(net.named_parameters()):
            key = '%s_gproj:%s' % (tag, k)
            if 'f64_' + key not in d.files:
                assert p.grad is None or not p.requires_grad, k
                continue
            mine = grad_projections(p.grad.detach().double().cpu().numpy(), cfg['seed'] + (10 if tag == 'G' else 11),
                                    i, cfg['proj'])
            p64, p32 = d['f64_' + key], d['f32_' + key]
            err, base, norm = (np.linalg.norm(mine - p64), np.linalg.norm(p32 - p64), np.linalg.norm(p64))
            bound = FACTOR * base + FLOOR * max(norm, 1e-30)
            errs.append(err / bound)
            if err > bound:
                fails.append((tag, k, 'err %.3e bound %.3e (ref f32 %.3e, |proj| %.3e)' % (err, bound, base, norm)))
        print('%s: %d parameter gradients, worst at %.1f %% of its bound, median %.1f %%' % (
            tag, len(errs), 100 * max(errs), 100 * float(np.median(errs))))
        worst = max(worst, max(errs))
    for f in [f for f in d.files if f.startswith('f64_log:')]:
        key = f[len('f64_log:'):]
        mine = np.array(model.log_dict[key], dtype=np.float64)
        ref64, ref32 = d[f], d['f32_log:' + key]
        assert mine.shape == ref64.shape, key
        scale = None
        if key in D_DIFFERENCES:
            scale = 2 * (np.linalg.norm(d['f64_log:D_real'][:, 1]) + np.linalg.norm(d['f64_log:D_fake'][:, 1]))
        ok, msg, r = _close(mine[:, 1], ref32[:, 1], ref64[:, 1], scale)
        print('log %-24s %s' % (key, msg))
        worst = max(worst, r)
        if not ok:
            fails.append(('log', key, msg))
    for k, v in model.netD.state_dict().items():
        if 'running' in k:
            ok, msg, r = _close(v.double().cpu().numpy(), d['f32_Dbuf:' + k], d['f64_Dbuf:' + k])
            worst = max(worst, r)
            if not ok:
                fails.append(('D buffer', k, msg))
    print('worst quantity at %.1f %% of its bound' % (100 * worst))
    assert not fails, fails


def _proj(v, seed, idx, k):
    g = np.asarray(v, dtype=np.float64).ravel()
    return np.random.default_rng([seed, idx]).standard_normal((k, g.size)) @ g


@pytest.mark.parametrize('precision', ['x3', 'f32'])
def test_c5_z_gradients_at_production_grid(gpu_device, precision):
    """Config 5: the latent RRDB-23 + CEM in eval mode (pre-pad) with the reference-made learned 13×13 kernel, generator
    frozen, B=8 × 128² LR; dL/dZ, dL/dLR and the output of images 0 and 7 against the REFERENCE's autograd in float64
    and float32 (tests/golden/make_golden.py c5grid), through seeded random projections."""
    import esr_amd
    from esr_amd import CEMnet as C
    from esr_amd import engine
    from oracle.recipe import seeded_inputs, seeded_params
    d = np.load(os.path.join(HERE, 'golden', 'grid_c5_zgrad.npz'))
    cfg = json.loads(str(d['cfg']))
    B, h, K = cfg['B'], cfg['h'], cfg['proj']
    net = esr_amd.RRDBNet(3, 3, 64, cfg['nb'], latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=d['kernel']).WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    params = seeded_params([(n, tuple(v.shape)) for n, v in sd.items()], cfg['seed'], w_scale=cfg['w_scale'])
    model.load_state_dict({n: torch.from_numpy(v) for n, v in params.items()}, strict=False)
    model = model.to(gpu_device)
    model.eval()
    engine.set_precision(model, precision)
    for q in model.parameters():
        q.requires_grad = False
    lr, z = seeded_inputs(cfg['seed'] + 1, (B, 3, h, h), (B, 3, 4 * h, 4 * h), z_mode='pixel')
    R = np.random.default_rng(cfg['seed'] + 2).standard_normal((B, 3, 4 * h, 4 * h)).astype(np.float32)
    zt = torch.from_numpy(z).to(gpu_device).requires_grad_(True)
    lt = torch.from_numpy(lr).to(gpu_device).requires_grad_(True)
    out = model(torch.cat([zt.view(B, 48, h, h), lt], 1))
    (out * torch.from_numpy(R).to(gpu_device)).sum().backward()
    fails, worst = [], 0.0
    for i in cfg['images']:
        for name, v in (('dz', zt.grad[i]), ('dlr', lt.grad[i]), ('out', out.detach()[i])):
            mine = _proj(v.double().cpu().numpy(), cfg['seed'] + {'dz': 10, 'dlr': 11, 'out': 12}[name], i, K)
            p64, p32 = d['f64_%s_proj:%d' % (name, i)], d['f32_%s_proj:%d' % (name, i)]
            err, base, norm = np.linalg.norm(mine - p64), np.linalg.norm(p32 - p64), np.linalg.norm(p64)
            if name == 'out':  # forward: the north_star bar, normwise-equivalent on the projections
                bound = 1e-5 * norm
            else:
                bound = FACTOR * base + FLOOR * norm
            worst = max(worst, err / bound)
            print('image %d %-4s err %.3e  bound %.3e  (%.1f %%; ref f32 %.3e, |proj| %.3e)' % (
                i, name, err, bound, 100 * err / bound, base, norm))
            if err > bound:
                fails.append((i, name, err, bound))
    assert not fails, fails
