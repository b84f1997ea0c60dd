"""GPU parity of the training path: HIP forward (x3 by default, or exact fp32) with retained activations + hand-written
backward (exact fp32)
against the reference's own training gradients (golden) and the oracle's autograd (all parameters).
Forward outputs: normwise 1e-5.  Gradients: conftest.grad_parity — relative L2 error against the float64 oracle within
5× that of the reference's own fp32 evaluation (floor 1e-4, a tenth of the 1e-3 bar; an indexing or layout bug
shows as O(1e-1) errors), which is robust to LeakyReLU kink flips."""
import numpy as np
import pytest
import torch

from conftest import fixture_input, fixture_params, fixture_upscale, golden, golden_names, grad_parity, normwise_rel, oracle_grads

import esr_amd
from esr_amd import CEMnet as C
from oracle import esr_oracle as O
from oracle.recipe import seeded_inputs, seeded_params

pytestmark = pytest.mark.gpu


def _model(nb, latent, params, dev, sf=4):
    net = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0, upscale=sf)
    model = C.CEMnet(C.Get_CEM_Config(sf)).WrapArchitecture_PyTorch(net)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    return model.to(dev).train(True)


@pytest.mark.parametrize('name', golden_names('grad_'))
def test_training_gradients_vs_reference_golden(gpu_device, name):
    d = golden(name)
    _, params = fixture_params(d)
    sf = fixture_upscale(d)  # ×4, and ×2 (grad_x2_*: one upconv)
    model = _model(int(d['nb']), bool(int(d['latent'])), params, gpu_device, sf)
    out = model(fixture_input(d).to(gpu_device))
    assert normwise_rel(out.detach().cpu(), d['out']) < 1e-5
    (out * torch.from_numpy(d['R']).to(gpu_device)).sum().backward()
    exact = oracle_grads(params, d['lr'], d['z'] if 'z' in d.files else None, d['R'], int(d['nb']),
                         bool(int(d['latent'])), O.cem_design(sf), False, torch.float64, sf=sf)
    named = dict(model.named_parameters())
    for k in [f[len('grad:'):] for f in d.files if f.startswith('grad:')]:
        g = named['generated_image_model.' + k].grad
        assert g is not None, k
        ok, msg = grad_parity(g.cpu(), exact['param:' + k], d['grad:' + k])
        assert ok, (k, msg)


@pytest.mark.parametrize('precision', ['x3', 'f32'])
@pytest.mark.parametrize('latent', [False, True])
def test_all_parameter_gradients_vs_oracle(gpu_device, latent, precision):
    """Every parameter gradient of a training step, with the forward in x3 (default: the backward reads split-f16
    activations) and in exact fp32."""
    from esr_amd import engine
    nb = 2
    net = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], 51, w_scale=0.7)
    model = _model(nb, latent, params, gpu_device)
    engine.set_precision(model, precision)
    B, h, w = 2, 10, 14
    lr, z = seeded_inputs(52, (B, 3, h, w), (B, 3, 4 * h, 4 * w) if latent else None, z_mode='pixel')
    x = torch.from_numpy(lr)
    if latent:
        x = torch.cat([torch.from_numpy(z).reshape(B, 48, h, w), x], 1)
    R = torch.from_numpy(np.random.default_rng(53).standard_normal((B, 3, 4 * h, 4 * w)).astype(np.float32))
    out = model(x.to(gpu_device))
    (out * R.to(gpu_device)).sum().backward()
    P = O.strip_prefix(params)
    with torch.no_grad():
        ref = O.sr_forward(x, P, nb, latent, O.cem_design(4), pre_pad=False)
    assert normwise_rel(out.detach().cpu(), ref) < 1e-5
    exact, base = (oracle_grads(params, lr, z, R, nb, latent, O.cem_design(4), False, dt)
                   for dt in (torch.float64, torch.float32))
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        k = 'param:' + n[len('generated_image_model.'):]
        ok, msg = grad_parity(p.grad.cpu(), exact[k], base[k])
        assert ok, (n, msg)


def test_training_step_is_deterministic(gpu_device):
    d = golden('grad_plain_nb1')
    _, params = fixture_params(d)
    grads = []
    for _ in range(2):
        model = _model(1, False, params, gpu_device)
        out = model(fixture_input(d).to(gpu_device))
        (out * torch.from_numpy(d['R']).to(gpu_device)).sum().backward()
        grads.append([p.grad.clone() for p in model.parameters() if p.requires_grad])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize('nb,latent', [(1, False), (2, True)])
def test_side_stream_weight_gradients_bitwise(gpu_device, nb, latent):
    """Weight gradients on the second stream (train_engine.WGRAD_STREAM, overlapping the data-gradient chain) give
    the same parameter gradients, bit for bit, as the one-stream backward, eagerly and through the captured HIP graphs
    (calls 2 and 3), in x3 and in exact fp32."""
    from esr_amd import engine, train_engine as TE
    from oracle.recipe import seeded_inputs, seeded_params
    B, h, w = 2, 12, 16
    net = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    sd = net.state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], 91, w_scale=0.5)
    lr, z = seeded_inputs(92, (B, 3, h, w), (B, 3, 4 * h, 4 * w), z_mode='pixel')
    x = torch.from_numpy(lr)
    if latent:
        x = torch.cat([torch.from_numpy(z).view(B, 48, h, w), x], 1)
    R = torch.from_numpy(np.random.default_rng(93).standard_normal((B, 3, 4 * h, 4 * w)).astype(np.float32))
    prev = TE.WGRAD_STREAM
    try:
        for prec in ('x3', 'f32'):
            runs = []
            for side in (True, False):
                TE.WGRAD_STREAM = side
                m = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled' if latent else None,
                                    num_latent_channels=3 if latent else 0)
                m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
                m = m.to(gpu_device)
                engine.set_precision(m, prec)
                calls = []
                for _ in range(3):  # eager, capture, replay
                    m.zero_grad()
                    (m(x.to(gpu_device)) * R.to(gpu_device)).sum().backward()
                    calls.append([q.grad.clone() for q in m.parameters()])
                runs.append(calls)
            for c in range(3):
                for a, b in zip(runs[0][c], runs[1][c]):
                    assert torch.equal(a, b), (prec, c)
    finally:
        TE.WGRAD_STREAM = prev


def test_optimize_parameters_training_step(gpu_device):
    """SRRaGANModel.optimize_parameters on the HIP generator: D step (WGAN-GP) every step, G step from step 1 on;
    both networks move, losses are finite, the generator output keeps the reference shape contract."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location('bench_train', os.path.join(os.path.dirname(__file__), '..',
                                                                              'bench_train.py'))
    bt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bt)
    from esr_amd.SRRaGAN_model import SRRaGANModel

    class A:
        batch, lr_size, nb, latent = 2, 40, 1, True
    torch.manual_seed(0)
    model = SRRaGANModel(bt.make_opt(A), device=gpu_device)
    g0 = [p.detach().clone() for p in model.netG.parameters() if p.requires_grad]
    d0 = [p.detach().clone() for p in model.netD.parameters()]
    data = {'LR': torch.rand(2, 3, 40, 40, device=gpu_device), 'HR': torch.rand(2, 3, 160, 160, device=gpu_device)}
    steps = []
    for _ in range(3):
        model.feed_data(data)
        model.optimize_parameters()
        steps.append(model.generator_step)
    assert steps == [False, True, True]
    assert tuple(model.fake_H.shape) == (2, 3, 80, 80)
    assert any(not torch.equal(a, b) for a, b in zip(g0, [p for p in model.netG.parameters() if p.requires_grad]))
    assert any(not torch.equal(a, b) for a, b in zip(d0, model.netD.parameters()))
    for k in ('l_d_real', 'l_d_fake', 'l_d_gp', 'l_g_gan', 'l_g_range'):
        assert model.log_dict[k] and np.isfinite(model.log_dict[k][-1][1]), k
    model.test()
    assert tuple(model.fake_H.shape) == (2, 3, 160, 160)


@pytest.mark.parametrize('name', golden_names('zgrad_'))
def test_z_gradients_vs_reference_golden(gpu_device, name):
    """Z optimisation (Z_optimization.py:545-630): generator frozen, gradient w.r.t. the model input only —
    replicate pre-pad adjoint (eval), bilinear ↓4 adjoint, Z slots of every conv, CEM's LR path."""
    d = golden(name)
    _, params = fixture_params(d)
    sf = fixture_upscale(d)  # ×4, and ×2 (zgrad_x2_*)
    net = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled', num_latent_channels=3, upscale=sf)
    cem = C.CEMnet(C.Get_CEM_Config(sf), upscale_kernel=d['kernel'] if 'kernel' in d.files else None)
    model = cem.WrapArchitecture_PyTorch(net)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    model = model.to(gpu_device).train(str(d['cem_mode']) == 'train')
    for p in model.parameters():
        p.requires_grad = False
    z = torch.from_numpy(d['z']).to(gpu_device).requires_grad_(True)
    lr = torch.from_numpy(d['lr']).to(gpu_device).requires_grad_(True)
    B, _, h, w = lr.shape
    out = model(torch.cat([z.view(B, 3 * sf * sf, h, w), lr], 1))
    assert normwise_rel(out.detach().cpu(), d['out']) < 1e-5
    (out * torch.from_numpy(d['R']).to(gpu_device)).sum().backward()
    design = O.cem_design(sf, d['kernel'] if 'kernel' in d.files else None)
    exact = oracle_grads(params, d['lr'], d['z'], d['R'], 1, True, design, str(d['cem_mode']) == 'eval',
                         torch.float64, want_params=False, sf=sf)
    for g, k in ((z.grad, 'dz'), (lr.grad, 'dlr')):
        ok, msg = grad_parity(g.cpu(), exact[k], d[k])
        assert ok, (k, msg)


# Gradient floor of conftest.grad_parity for an x3 forward: its activations carry ~2^-21 relative rounding (fp32:
# 2^-24), so a LeakyReLU pre-activation within that of 0 takes the other slope about 8x as often as in an fp32 forward.
# In the eval-mode CEM pre-pad margin (a replicated border: whole lines of equal pre-activations) such flips moved
# weight gradients by up to 7.6e-4 L2, so parameter gradients with pre-pad use the exact-fp32 forward (train_engine);
# the x3 cases below are held to 5e-4, the fp32 ones to the default 1e-4, all under the 1e-3 parity bar (an indexing
# bug shows as O(1e-1)).
X3_GRAD_FLOOR = 5e-4


@pytest.mark.parametrize('precision', ['x3', 'f32'])
@pytest.mark.parametrize('mode', ['eval', 'train'])
def test_input_and_parameter_gradients_together_vs_oracle(gpu_device, mode, precision):
    """Both gradient kinds in one backward (nb=2, latent, pixel Z) against the oracle's autograd."""
    from esr_amd import engine
    nb = 2
    net = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net)
    params = seeded_params([(k, tuple(v.shape)) for k, v in model.state_dict().items()], 61, w_scale=0.7)
    model = _model(nb, True, params, gpu_device).train(mode == 'train')
    engine.set_precision(model, precision)
    floor = X3_GRAD_FLOOR if precision == 'x3' else 1e-4
    B, h, w = 2, 12, 10
    lr, z = seeded_inputs(62, (B, 3, h, w), (B, 3, 4 * h, 4 * w), z_mode='pixel')
    zt = torch.from_numpy(z).to(gpu_device).requires_grad_(True)
    out = model(torch.cat([zt.view(B, 48, h, w), torch.from_numpy(lr).to(gpu_device)], 1))
    R = torch.from_numpy(np.random.default_rng(63).standard_normal(tuple(out.shape)).astype(np.float32))
    (out * R.to(gpu_device)).sum().backward()
    exact, base = (oracle_grads(params, lr, z, R, nb, True, O.cem_design(4), mode == 'eval', dt)
                   for dt in (torch.float64, torch.float32))
    ok, msg = grad_parity(zt.grad.cpu(), exact['dz'], base['dz'], floor=floor)
    assert ok, msg
    for n, p in model.named_parameters():
        if p.requires_grad:
            k = 'param:' + n[len('generated_image_model.'):]
            ok, msg = grad_parity(p.grad.cpu(), exact[k], base[k], floor=floor)
            assert ok, (n, msg)


@pytest.mark.parametrize('variant', [0, 1, 'x3', 'x3_dsplit', 'x3_dsplit_reg'])
@pytest.mark.parametrize('cin,in_cp,cout,dout_cp,dout_coff,up2,B,H,W,splits', [
    (64, 64, 32, 192, 64, 0, 2, 20, 40, 7),      # RDB growth conv: dout a channel slice of a concat buffer
    (72, 80, 64, 64, 0, 0, 3, 13, 33, 5),        # latent-slot input, cout 64, ragged tiles
    (64, 64, 64, 72, 8, 1, 2, 24, 64, 16),       # upconv: nearest x2 input read on the fly
    (64, 64, 3, 8, 0, 0, 1, 17, 35, 3),          # HR_conv1: cout 3 (scalar output-gradient loads)
    (200, 200, 32, 32, 0, 0, 2, 8, 32, 1),       # partial last input chunk (cin_pad 224), one split
    (64, 64, 32, 36, 2, 0, 2, 9, 31, 4),         # unaligned output-gradient pitch / offset
])
def test_weight_gradient_kernels_vs_float64(gpu_device, variant, cin, in_cp, cout, dout_cp, dout_coff, up2, B, H, W,
                                            splits, request):
    """esr_conv3x3_wgrad (both fp32 kernels, and the x3 kernel on split-f16 activations) + esr_wgrad_reduce against
    torch.nn.grad.conv2d_weight in float64.  The x3 kernel splits the output gradient per pixel tile after a
    power-of-two scaling; here the output gradient is ~2^-30 (a realistic loss-gradient magnitude, far below f16's
    range) and its magnitude changes by 2^3 steps from one 8-row tile / image to the next, so that tiles take
    different scales (the accumulator is rescaled between them) and every tile still counts in the norm.
    x3_dsplit: the output gradient split-f16 at one scale S (the x3 backward's layout, flags bit 8) on the LDS-DMA
    kernel (wgrad3d); x3_dsplit_reg: the same on the register-staged x3 kernel.  Variants 0 and x3_dsplit_reg run on
    the ablation library (the product library's choices are 1 / the LDS-DMA kernel)."""
    import ctypes
    from esr_amd import _lib
    ablation = variant in (0, 'x3_dsplit_reg')
    lib = request.getfixturevalue('ablation_lib') if ablation else _lib.load()
    g = torch.Generator().manual_seed(cin * 7 + cout)
    Hi, Wi = (H // 2, W // 2) if up2 else (H, W)
    x = torch.randn(B, cin, Hi, Wi, generator=g)
    dy = torch.randn(B, cout, H, W, generator=g)
    xin = torch.zeros(B, Hi + 2, Wi + 2, in_cp)
    xin[:, 1:-1, 1:-1, :cin] = x.permute(0, 2, 3, 1)
    dbuf = torch.randn(B, H + 2, W + 2, dout_cp, generator=g)  # junk around the slice must be ignored
    x3 = str(variant).startswith('x3')
    dsplit = str(variant).startswith('x3_dsplit')
    if dsplit and (cout % 8 or dout_cp % 8 or dout_coff % 8):
        pytest.skip('a split-f16 output gradient needs 8-channel groups')
    if x3:
        if cin % 8 or in_cp % 8:
            pytest.skip('split-f16 activations need 8-channel groups')
        tile = torch.arange(H).view(1, H) // 8 + torch.arange(B).view(B, 1)
        dy = dy * torch.exp2(-30.0 + 3.0 * (tile % 5 - 2)).view(B, 1, H, 1)  # 2^-36 .. 2^-24 by tile
    dbuf[:, 1:-1, 1:-1, dout_coff:dout_coff + cout] = dy.permute(0, 2, 3, 1)
    flags = up2
    S = 1.0
    if x3:
        from esr_amd import engine as E
        xin = E.to_split(xin)
        x = E.from_split(E.to_split(x.permute(0, 2, 3, 1).contiguous())).permute(0, 3, 1, 2)  # the values it holds
        flags = up2 | 6
    if dsplit:
        S = 2.0 ** 34  # S·dy: largest |S·dy| ~2^12, the smallest tiles' values ~2^-2
        dbuf = E.to_split(dbuf * S)
        dy = E.from_split(E.to_split((dy * S).permute(0, 2, 3, 1).contiguous())).permute(0, 3, 1, 2) / S
        flags |= 8
    cin_pad, cout_pad = 32 * ((cin + 31) // 32), 64 if cout > 32 else 32
    n = 9 * cin_pad * cout_pad + cout_pad
    xin, dbuf = xin.to(gpu_device), dbuf.to(gpu_device)
    partial = torch.full((splits * n,), float('nan'), device=gpu_device)
    out = torch.empty(n, device=gpu_device)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if ablation:
        lib.esr_wgrad_set_kernel(variant if not x3 else 1)
        lib.esr_wgrad3_set_dma(0 if variant == 'x3_dsplit_reg' else 1)
    try:
        _lib.check(lib.esr_conv3x3_wgrad(xin.data_ptr(), in_cp, cin, flags, dbuf.data_ptr(), dout_cp, dout_coff, cout,
                                         B, H, W, splits, partial.data_ptr(), st), 'wgrad')
        _lib.check(lib.esr_wgrad_reduce(partial.data_ptr(), splits, n, 1.0 / S, out.data_ptr(), st), 'reduce')
        torch.cuda.synchronize()
    finally:
        if ablation:
            lib.esr_wgrad_set_kernel(1)
            lib.esr_wgrad3_set_dma(1)
    out = out.cpu().double()
    xr = x.double()
    if up2:
        xr = xr.repeat_interleave(2, 2).repeat_interleave(2, 3)
    ref_w = torch.nn.grad.conv2d_weight(xr, (cout, cin, 3, 3), dy.double(), padding=1)  # [co][ci][ky][kx]
    got_w = out[:9 * cin_pad * cout_pad].view(3, 3, cin_pad, cout_pad)[:, :, :cin, :cout].permute(3, 2, 0, 1)
    assert normwise_rel(got_w, ref_w) < 1e-5
    assert normwise_rel(out[9 * cin_pad * cout_pad:][:cout], dy.double().sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize('latent', [False, True])
def test_graph_replay_equals_eager(gpu_device, latent):
    """The HIP-graph replay of the training forward/backward (captured on the second call of a shape) gives bitwise the
    eager results over several optimiser steps (the parameter repack runs outside the graph), for parameter and
    input gradients."""
    from esr_amd import train_engine as T
    from oracle.recipe import seeded_params
    net0 = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled' if latent else None,
                           num_latent_channels=3 if latent else 0)
    shapes = [(k, tuple(v.shape)) for k, v in C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net0)
              .state_dict().items() if 'Filter' not in k]
    params = seeded_params(shapes, 61, w_scale=0.5)
    lr, z = seeded_inputs(62, (2, 3, 12, 16), (2, 3, 48, 64) if latent else None)
    x = torch.from_numpy(lr)
    if latent:
        x = torch.cat([torch.from_numpy(z).reshape(2, 48, 12, 16), x], 1)
    R = torch.from_numpy(np.random.default_rng(63).standard_normal((2, 3, 48, 64)).astype(np.float32))
    runs = {}
    prev = T.USE_GRAPHS
    try:
        for graphs in (False, True):
            T.USE_GRAPHS = graphs
            model = _model(1, latent, params, gpu_device)
            opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=1e-3)
            xin = x.to(gpu_device).requires_grad_(True)
            rec = []
            for _ in range(4):
                opt.zero_grad()
                xin.grad = None
                out = model(xin)
                (out * R.to(gpu_device)).sum().backward()
                rec.append([out.detach().clone(), xin.grad.clone()] +
                           [p.grad.clone() for p in model.parameters() if p.requires_grad])
                opt.step()
            runs[graphs] = rec
    finally:
        T.USE_GRAPHS = prev
    for step, (a, b) in enumerate(zip(runs[False], runs[True])):
        for i, (u, v) in enumerate(zip(a, b)):
            assert torch.equal(u, v), (step, i)


@pytest.mark.parametrize('mode', ['eval', 'train'])
def test_frozen_generator_input_gradient_x3_forward(gpu_device, mode):
    """Generator frozen, input gradient only (the Z-optimisation case): the forward runs in x3 and the backward reads
    its split-f16 activations (LeakyReLU masks).  Output and input gradient against the float64 oracle, within 5x the
    oracle's own fp32 error (floor 1e-4); eager, captured and replayed runs bitwise equal, for x3 and for the
    exact-fp32 forward.  (The fp32 run is not held to the oracle here: at this seed in eval mode one LeakyReLU
    pre-activation in the replicate-padded margin lies within fp32 rounding of 0 and takes the other slope, an input
    gradient L2 difference of 1.7e-4 collected by the border pixels — conftest.grad_parity's kink case.)"""
    from esr_amd import engine
    from oracle.recipe import seeded_params
    net0 = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    shapes = [(k, tuple(v.shape)) for k, v in C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net0)
              .state_dict().items() if 'Filter' not in k]
    params = seeded_params(shapes, 81, w_scale=0.5)
    lr, z = seeded_inputs(82, (2, 3, 12, 12), (2, 3, 48, 48))
    x = torch.cat([torch.from_numpy(z).reshape(2, 48, 12, 12), torch.from_numpy(lr)], 1)
    res = {}
    for prec in ('x3', 'f32'):
        model = _model(1, True, params, gpu_device).train(mode == 'train')
        engine.set_precision(model, prec)
        for p in model.parameters():
            p.requires_grad = False
        out_shape = model(x.to(gpu_device)).shape
        R = torch.from_numpy(np.random.default_rng(83).standard_normal(out_shape).astype(np.float32))
        outs = []
        for _ in range(3):  # eager, graph capture, replay
            xin = x.to(gpu_device).requires_grad_(True)
            out = model(xin)
            (out * R.to(gpu_device)).sum().backward()
            outs.append((out.detach().cpu(), xin.grad.cpu()))
        for o, g in outs[1:]:
            assert torch.equal(o, outs[0][0]) and torch.equal(g, outs[0][1])
        res[prec] = outs[0]
    P = O.strip_prefix(params)
    ref = {}
    for dt in (torch.float64, torch.float32):
        xr = x.clone().to(dt).requires_grad_(True)
        Pd = {k: torch.as_tensor(v).to(dt) for k, v in P.items()}
        out = O.sr_forward(xr, Pd, 1, True, O.cem_design(4), pre_pad=mode == 'eval')
        (out * R.to(dt)).sum().backward()
        ref[dt] = (out.detach(), xr.grad)
    for prec in ('x3', 'f32'):
        assert normwise_rel(res[prec][0], ref[torch.float64][0]) < 1e-5, prec
    ok, msg = grad_parity(res['x3'][1], ref[torch.float64][1], ref[torch.float32][1])
    assert ok, msg


def test_fused_gradient_amax_bitwise(gpu_device):
    """The x3 backward with each RRDB's gradient max taken by the previous RRDB's closing add (esr_axpby_gs_amax,
    train_engine.AMAX_FUSED) gives the same parameter and input gradients, bit for bit, as a separate esr_grad_amax
    pass (max is exact in any order)."""
    from esr_amd import engine, train_engine as TE
    from oracle.recipe import seeded_inputs, seeded_params
    B, h, w, nb = 2, 12, 16, 3
    kw = dict(latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    sd = esr_amd.RRDBNet(3, 3, 64, nb, **kw).state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], 95, w_scale=0.5)
    lr, z = seeded_inputs(96, (B, 3, h, w), (B, 3, 4 * h, 4 * w), z_mode='pixel')
    x = torch.cat([torch.from_numpy(z).view(B, 48, h, w), torch.from_numpy(lr)], 1)
    R = torch.from_numpy(np.random.default_rng(97).standard_normal((B, 3, 4 * h, 4 * w)).astype(np.float32))
    prev = TE.AMAX_FUSED
    try:
        runs = []
        for fused in (True, False):
            TE.AMAX_FUSED = fused
            m = esr_amd.RRDBNet(3, 3, 64, nb, **kw)
            m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
            m = m.to(gpu_device)
            engine.set_precision(m, 'x3')
            xi = x.to(gpu_device).requires_grad_()
            (m(xi) * R.to(gpu_device)).sum().backward()
            runs.append([q.grad.clone() for q in m.parameters()] + [xi.grad.clone()])
        for a, b in zip(*runs):
            assert torch.equal(a, b)
    finally:
        TE.AMAX_FUSED = prev


@pytest.mark.parametrize('B,H,W', [(2, 9, 13), (1, 3, 300)])
def test_axpby_rows_kernel_bitwise(gpu_device, ablation_lib, B, H, W):
    """esr_axpby_gs on the row-walking kernel with 4 items in flight per thread (product, knob 2) and with one (knob
    1) against the one-thread-per-8-channel-group kernel (knob 0): the same results, bit for bit, in every operand form
    the x3 backward uses (fp32 / split-f16 in and out, with and without x2, an overflow flag), including rows whose
    item count is not a multiple of the 4 x 256 a block covers per pass (W = 13 and W = 300)."""
    import ctypes
    from esr_amd import engine
    lib = ablation_lib
    cp = 72
    g = torch.Generator(device='cpu').manual_seed(5)
    amax = torch.tensor([0.0], device=gpu_device)
    amax.fill_(37.5)
    amax_u = amax.view(torch.int32)
    f1 = torch.randn(B, H + 2, W + 2, cp, generator=g).to(gpu_device)
    f2 = torch.randn(B, H + 2, W + 2, cp, generator=g).to(gpu_device)
    s2 = engine.to_split(torch.randn(B, H + 2, W + 2, 32, generator=g).to(gpu_device) * 100)  # 32 ch, 32 floats
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    forms = [  # (o_split, x1, x1_split, x2, x2_split, o_cp, C)
        (0, f1, 0, f2, 0, cp, 64), (0, f1, 0, s2, 1, cp, 32), (1, f1, 0, None, 0, cp, 64), (0, s2, 1, None, 0, cp, 32),
        (0, f1, 0, None, 0, cp, 8)]
    try:
        for o_split, x1, x1s, x2, x2s, o_cp, C in forms:
            outs = []
            for rows in (2, 1, 0):
                lib.esr_axpby_set_rows(rows)
                out = torch.zeros(B, H + 2, W + 2, o_cp, device=gpu_device)
                ovf = torch.zeros(1, dtype=torch.int32, device=gpu_device)
                _lib_check = lib.esr_axpby_gs(out.data_ptr(), o_cp, 8, o_split, 0.7, x1.data_ptr(), x1.shape[-1], 0,
                                              x1s, -1.3, x2.data_ptr() if x2 is not None else None,
                                              x2.shape[-1] if x2 is not None else 0, 0, x2s, C, B, H, W,
                                              amax_u.data_ptr(), ovf.data_ptr(), st)
                assert _lib_check == 0
                torch.cuda.synchronize()
                outs.append((out, ovf))
            for k in (1, 2):
                assert torch.equal(outs[0][0], outs[k][0]) and torch.equal(outs[0][1], outs[k][1]), (o_split, x1s, x2s,
                                                                                                    C, k)
    finally:
        lib.esr_axpby_set_rows(2)


@pytest.mark.parametrize('latent', [False, True])
def test_hr1_data_gradient_on_first_conv_kernel(gpu_device, latent):
    """HR_conv1's data gradient on esr_dfirst_fwd_padded (train_engine.HR1_DFIRST: exact fp32 on the VALU) against the
    fp32 MFMA conv it replaces: every parameter gradient and the input gradient agree to fp32 rounding (1e-5)."""
    from esr_amd import engine, train_engine as TE
    from oracle.recipe import seeded_inputs, seeded_params
    B, h, w, nb = 2, 12, 16, 1
    kw = dict(latent_input='all_layers_HR_downscaled' if latent else None, num_latent_channels=3 if latent else 0)
    sd = esr_amd.RRDBNet(3, 3, 64, nb, **kw).state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], 98, w_scale=0.5)
    lr, z = seeded_inputs(99, (B, 3, h, w), (B, 3, 4 * h, 4 * w), z_mode='pixel')
    x = torch.from_numpy(lr)
    if latent:
        x = torch.cat([torch.from_numpy(z).view(B, 48, h, w), x], 1)
    R = torch.from_numpy(np.random.default_rng(100).standard_normal((B, 3, 4 * h, 4 * w)).astype(np.float32))
    prev = TE.HR1_DFIRST
    try:
        runs = []
        for on in (True, False):
            TE.HR1_DFIRST = on
            m = esr_amd.RRDBNet(3, 3, 64, nb, **kw)
            m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
            m = m.to(gpu_device)
            engine.set_precision(m, 'f32')
            xi = x.to(gpu_device).requires_grad_()
            (m(xi) * R.to(gpu_device)).sum().backward()
            runs.append(torch.cat([q.grad.reshape(-1) for q in m.parameters()] + [xi.grad.reshape(-1)]).cpu())
        assert normwise_rel(runs[0], runs[1]) < 1e-5
    finally:
        TE.HR1_DFIRST = prev
