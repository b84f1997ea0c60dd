"""Production-grid parity checks shared by tests/test_gpu_grid.py and bench.py's reference-check leg (TEST
INFRASTRUCTURE: reference-made fixtures tests/golden/grid_c3_train.npz and grid_c5_zgrad.npz; the seeded weights and
inputs come from oracle/recipe.py's NumPy recipe).

Each check returns {'ok': bool, 'worst_frac_of_bound': float, 'fails': [...], 'lines': [...]} where a quantity's
bound is the reference's own float32 distance to its float64 run × 5 plus a floor of 1e-4 of the quantity's scale
(conftest.grad_parity's yardstick), evaluated through K seeded random projections where the fixture cannot hold the
full float64 tensors.  Config 3: the float32 distance is the largest over the plain reference run and its
rounding-perturbed runs (f32p*, make_golden_train.py c3p), as in the training-loop test; the bound of the plain run
alone is reported beside it ('worst_frac_of_single_run_bound') and capped at SINGLE_RUN_CEILING."""
import contextlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (HERE, os.path.join(HERE, 'golden'), os.path.dirname(HERE)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FACTOR, FLOOR = 5.0, 1e-4
# config 3 also caps the error against the plain single float32 run's bound, so that the wider ensemble yardstick cannot
# hide a drift (round 5: x3 87.0 %, f32 under the three upsampler folds 80.7 / 104.5 / 80.9 % of it)
SINGLE_RUN_CEILING = 1.25


def _proj(v, seed, idx, k):
    g = np.asarray(v, dtype=np.float64).ravel()
    return np.random.default_rng([seed, idx]).standard_normal((k, g.size)) @ g


def _result(fails, worst, lines, worst_single=None):
    r = {'ok': not fails, 'worst_frac_of_bound': round(float(worst), 4), 'fails': fails, 'lines': lines}
    if worst_single is not None:
        r['worst_frac_of_single_run_bound'] = round(float(worst_single), 4)
    return r


def c3_training_step(dev, precision='x3', d_precision=None):
    """Config 3 (B=16 × 96² LR, RRDB-23, latent, CEM train mode, WGAN-GP): two optimize_parameters micro-steps against
    the reference's own run (tests/golden/make_golden_train.py c3); the step-1 gradient of every G and D parameter,
    the logs and the D BatchNorm buffers."""
    from test_gpu_train_loop import D_DIFFERENCES, _close, _f32s, _run_port
    from train_recipe import grad_projections
    from esr_amd import dconv
    d = np.load(os.path.join(HERE, 'golden', 'grid_c3_train.npz'))
    cfg = json.loads(str(d['cfg']))
    prev = dconv.PRECISION
    try:
        model, _, _, flags = _run_port(cfg, precision, dev, d_precision)
    finally:
        dconv.set_precision(prev)
    fails, worst, worst1, lines = [], 0.0, 0.0, []
    n_runs = len(_f32s(d, '%s_generator_step'))
    if not flags == list(d['f64_generator_step']) == list(d['f32_generator_step']):
        fails.append(('generator_step', flags))
    lines.append('yardstick: %d reference float32 run(s) (the plain run + %d rounding-perturbed ones, '
                 'make_golden_train.py c3p): bound = %g x the largest float32 distance to the float64 run + %g x |ref|; '
                 'the single-run bound (plain float32 run only) is printed beside it' % (n_runs, n_runs - 1, FACTOR,
                                                                                         FLOOR))
    for net, tag in ((model.netG, 'G'), (model.netD, 'D')):
        errs, errs1, names = [], [], []
        for i, (k, p) in enumerate(net.named_parameters()):
            key = '%s_gproj:%s' % (tag, k)
            if 'f64_' + key not in d.files:
                continue
            if p.grad is None:
                if 'Filter_OP' in k:  # the CEM filters: requires_grad=False at construction (CEMnet.py:134), so the
                    continue          # reference's optimizer_G leaves them out (SRRaGAN_model.py:207-211); their .grad
                    #                   there is a by-product of optimize_parameters re-enabling requires_grad (:468)
                fails.append((tag, k, 'no gradient'))
                continue
            mine = grad_projections(p.grad.detach().double().cpu().numpy(), cfg['seed'] + (10 if tag == 'G' else 11),
                                    i, cfg['proj'])
            p64 = d['f64_' + key]
            bases = [np.linalg.norm(v - p64) for v in _f32s(d, '%s_' + key)]
            err, base, norm = np.linalg.norm(mine - p64), max(bases), np.linalg.norm(p64)
            bound = FACTOR * base + FLOOR * max(norm, 1e-30)
            errs.append(err / bound)
            errs1.append(err / (FACTOR * bases[0] + FLOOR * max(norm, 1e-30)))
            names.append(k)
            if err > bound:
                fails.append((tag, k, 'err %.3e bound %.3e (ref f32 %.3e over %d runs, plain %.3e, |proj| %.3e)' % (
                    err, bound, base, len(bases), bases[0], norm)))
        order = np.argsort(errs)[::-1][:3]
        order1 = np.argsort(errs1)[::-1][:3]
        lines.append('%s: %d parameter gradients, worst at %.1f %% of its bound, median %.1f %% (worst: %s); single-run '
                     'bound: worst %.1f %% (%s)' % (
                         tag, len(errs), 100 * max(errs), 100 * float(np.median(errs)),
                         ', '.join('%s %.1f %%' % (names[j], 100 * errs[j]) for j in order), 100 * max(errs1),
                         ', '.join('%s %.1f %%' % (names[j], 100 * errs1[j]) for j in order1)))
        worst = max(worst, max(errs))
        worst1 = max(worst1, max(errs1))
    for f in [f for f in d.files if f.startswith('f64_log:')]:
        key = f[len('f64_log:'):]
        mine = np.array(model.log_dict[key], dtype=np.float64)
        ref64, ref32 = d[f], d['f32_log:' + key]
        if mine.shape != ref64.shape:
            fails.append(('log', key, 'shape %s vs %s' % (mine.shape, ref64.shape)))
            continue
        scale = None
        if key in D_DIFFERENCES:
            scale = 2 * (np.linalg.norm(d['f64_log:D_real'][:, 1]) + np.linalg.norm(d['f64_log:D_fake'][:, 1]))
        ok, msg, r = _close(mine[:, 1], [v[:, 1] for v in _f32s(d, '%s_log:' + key)], ref64[:, 1], scale)
        lines.append('log %-24s %s' % (key, msg))
        worst = max(worst, r)
        worst1 = max(worst1, _close(mine[:, 1], ref32[:, 1], ref64[:, 1], scale)[2])
        if not ok:
            fails.append(('log', key, msg))
    for k, v in model.netD.state_dict().items():
        if 'running' in k:
            mine = v.double().cpu().numpy()
            ok, msg, r = _close(mine, _f32s(d, '%s_Dbuf:' + k), d['f64_Dbuf:' + k])
            worst = max(worst, r)
            worst1 = max(worst1, _close(mine, d['f32_Dbuf:' + k], d['f64_Dbuf:' + k])[2])
            if not ok:
                fails.append(('D buffer', k, msg))
    if worst1 > SINGLE_RUN_CEILING:
        fails.append(('single-run bound', 'worst at %.1f %% of the plain float32 run\'s bound (ceiling %.0f %%)' % (
            100 * worst1, 100 * SINGLE_RUN_CEILING)))
    return _result(fails, worst, lines, worst1)


FOLDS = ('product', 'rowmajor', 'f64')


@contextlib.contextmanager
def upsampler_fold(name):
    """Runs the upsampler phases' folded weights (engine.fold_upconv_phase: nearest-×2 + 3×3 conv as four 2×2 convs,
    each phase tap a sum of 1, 2 or 4 of the 3×3 taps) summed in another legal order, exact-fp32 path only:
    'product' = the shipped x-major order (engine.fold_terms), 'rowmajor' = y-major sequential, 'f64' = the exactly
    rounded sum (profiles/r4_c3_fold_order.txt).  The order changes the folded weights by an ulp, which is the kind of
    change the config-3 yardstick has to tolerate."""
    from esr_amd import engine as E
    if name == 'product':
        yield
        return

    def fold(w, py, px, f):
        t = E.fold_term_images(w.detach().double() if name == 'f64' else w.detach(), py, px, f)
        if name == 'f64':
            return (((t[0] + t[1]) + t[2]) + t[3]).float()
        terms = E.fold_terms(py, px, f)
        out = torch.zeros_like(t[0])
        for a in range(2):
            for b in range(2):
                for (y, x) in sorted(terms[a][b]):  # row-major: y, then x
                    out[:, :, a, b] += w.detach()[:, :, y, x]
        return out
    refresh = E._Packed.refresh

    def fold_refresh(self):
        refresh(self)
        with torch.no_grad():
            for row, (j, f) in zip(self.up, E.up_stages(self.net)):
                w = self.net.model[j][1].weight
                for cw, (py, px) in zip(row, [(a, b) for a in range(f) for b in range(f)]):
                    cw.f32.copy_(E.pack_conv_weight(fold(w, py, px, f), list(range(64)), 64))
    E._Packed.refresh = fold_refresh
    try:
        yield
    finally:
        E._Packed.refresh = refresh


C5_FIXTURES = {'learned13': 'grid_c5_zgrad.npz', 'kgan': 'grid_c5_zgrad_kgan.npz'}


def c5_z_gradients(dev, precision='x3', kernel='kgan'):
    """Config 5 (latent RRDB-23 + CEM eval, generator frozen, B=8 × 128²): dL/dZ, dL/dLR and the output of images 0 and
    7 against the reference's autograd.  kernel 'kgan': the ×4 kernel of the reference's KernelGAN post-processing
    (post_process_k + analytic_kernel, 33×33 after kernel_shift; CEM margins 22 / 88, G at 172²; make_golden.py
    c5grid_kgan) — SURVEY §8's config-5 geometry; 'learned13': the 13×13 learned kernel of the CEM fixtures (margins
    13 / 52, G at 154²; make_golden.py c5grid)."""
    import esr_amd
    from esr_amd import CEMnet as C
    from esr_amd import engine
    from oracle.recipe import seeded_inputs, seeded_params
    d = np.load(os.path.join(HERE, 'golden', C5_FIXTURES[kernel]))
    cfg = json.loads(str(d['cfg']))
    B, h, K = cfg['B'], cfg['h'], cfg['proj']
    net = esr_amd.RRDBNet(3, 3, 64, cfg['nb'], latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=d['kernel']).WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    params = seeded_params([(n, tuple(v.shape)) for n, v in sd.items()], cfg['seed'], w_scale=cfg['w_scale'])
    model.load_state_dict({n: torch.from_numpy(v) for n, v in params.items()}, strict=False)
    model = model.to(dev)
    model.eval()
    engine.set_precision(model, precision)
    for q in model.parameters():
        q.requires_grad = False
    lr, z = seeded_inputs(cfg['seed'] + 1, (B, 3, h, h), (B, 3, 4 * h, 4 * h), z_mode='pixel')
    R = np.random.default_rng(cfg['seed'] + 2).standard_normal((B, 3, 4 * h, 4 * h)).astype(np.float32)
    zt = torch.from_numpy(z).to(dev).requires_grad_(True)
    lt = torch.from_numpy(lr).to(dev).requires_grad_(True)
    out = model(torch.cat([zt.view(B, 48, h, h), lt], 1))
    (out * torch.from_numpy(R).to(dev)).sum().backward()
    fails, worst, lines = [], 0.0, []
    for i in cfg['images']:
        for name, v in (('dz', zt.grad[i]), ('dlr', lt.grad[i]), ('out', out.detach()[i])):
            mine = _proj(v.double().cpu().numpy(), cfg['seed'] + {'dz': 10, 'dlr': 11, 'out': 12}[name], i, K)
            p64, p32 = d['f64_%s_proj:%d' % (name, i)], d['f32_%s_proj:%d' % (name, i)]
            err, base, norm = np.linalg.norm(mine - p64), np.linalg.norm(p32 - p64), np.linalg.norm(p64)
            # the output against the north_star bar's tenth (1e-4 relative on the projections); gradients as above
            bound = 1e-4 * norm if name == 'out' else FACTOR * base + FLOOR * norm
            worst = max(worst, err / bound)
            lines.append('image %d %-4s err %.3e  bound %.3e  (%.1f %%; ref f32 %.3e, |proj| %.3e)' % (
                i, name, err, bound, 100 * err / bound, base, norm))
            if err > bound:
                fails.append((i, name, err, bound))
    return _result(fails, worst, lines)
