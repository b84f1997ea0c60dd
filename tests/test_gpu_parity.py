"""GPU parity of the HIP path (libesr_amd via the esr_amd modules) against the reference's golden vectors and the CPU
oracle.  Tolerances (north_star: within 1e-3 relative fp32; SURVEY.md §8d normwise metric max|y-ref|/max|ref|):
  single conv / stencil vs float64 CPU:   1e-5   (fp32 FMA chains of ≤1800 terms)
  whole generator vs reference fixtures:  1e-4   (observed ~1e-6; the contract is 1e-3)
  full-size RRDB-23 + CEM vs oracle:      1e-3   (the north_star bar)
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import fixture_input, fixture_upscale, fixture_params, golden, golden_names, normwise_rel

import esr_amd
from esr_amd import CEMnet as C
from esr_amd import _lib, engine
from oracle import esr_oracle as O

pytestmark = pytest.mark.gpu


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _padded(B, H, W, cp, cin, dev, seed):
    g = torch.Generator().manual_seed(seed)
    buf = torch.zeros(B, H + 2, W + 2, cp)
    buf[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, generator=g) * 2 - 1
    if cp > cin:  # channels beyond cin hold garbage the kernel must not read
        buf[:, 1:-1, 1:-1, cin:] = 1e30
    return buf.to(dev)


def _nchw(buf, c0, c1):
    return buf[:, 1:-1, 1:-1, c0:c1].permute(0, 3, 1, 2).double().cpu()


@pytest.mark.parametrize('cin,cout,H,W', [(8, 64, 5, 7), (72, 32, 13, 37), (200, 64, 9, 33), (64, 3, 17, 31),
                                          (136, 32, 8, 32), (16, 64, 1, 1)])
def test_conv3x3_layer(gpu_device, cin, cout, H, W):
    lib = _lib.load()
    B = 2
    cp = cin + 8
    x = _padded(B, H, W, cp, cin, gpu_device, 1)
    g = torch.Generator().manual_seed(2)
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.1)
    b = (torch.rand(cout, generator=g) - 0.5)
    wp = engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 32 if cout <= 32 else 64)
    bd = b.to(gpu_device)
    out = torch.zeros(B, H + 2, W + 2, 72, device=gpu_device)
    res = _padded(B, H, W, 72, 72, gpu_device, 3)
    out2 = torch.zeros(B, H + 2, W + 2, 64, device=gpu_device)
    o = engine._conv_out(out, 72, 5, H, W, True, r1=res, r1_cp=72, r1_coff=1, s1=0.2, r2=res, r2_cp=72, r2_coff=2,
                         s2=0.5, out2=out2, out2_cp=64, out2_coff=0) if cout + 5 <= 72 else \
        engine._conv_out(out, 72, 0, H, W, True)
    _lib.check(lib.esr_conv3x3_fwd(x.data_ptr(), B, H, W, cp, cin, wp.data_ptr(), bd.data_ptr(), cout,
                                   ctypes.byref(o), _stream()), 'conv')
    torch.cuda.synchronize()
    ref = F.leaky_relu(F.conv2d(_nchw(x, 0, cin), w.double(), b.double(), padding=1), 0.2)
    if cout + 5 <= 72:
        ref = 0.5 * (0.2 * ref + _nchw(res, 1, 1 + cout)) + _nchw(res, 2, 2 + cout)
        assert normwise_rel(_nchw(out, 5, 5 + cout), ref) < 1e-5
        assert torch.equal(out2[:, 1:-1, 1:-1, :cout].cpu(), out[:, 1:-1, 1:-1, 5:5 + cout].cpu())
        assert torch.all(out[..., :5] == 0) and torch.all(out[..., 5 + cout:] == 0)
    else:
        assert normwise_rel(_nchw(out, 0, cout), ref) < 1e-5
    # halo untouched
    assert torch.all(out[:, 0] == 0) and torch.all(out[:, -1] == 0) and torch.all(out[:, :, 0] == 0)


@pytest.mark.parametrize('cin,cout,H,W', [(72, 32, 13, 37), (136, 64, 30, 70)])
def test_conv3x3_xcd_tile_map_bitwise(gpu_device, ablation_lib, cin, cout, H, W):
    """Exact-fp32 conv: XCD-grouped tile order (the product library) against row-major blockIdx order (the ablation
    library), bit for bit."""
    lib = _lib.load()
    B = 3
    cp = cin + 8
    x = _padded(B, H, W, cp, cin, gpu_device, 5)
    g = torch.Generator().manual_seed(6)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.1
    bd = (torch.rand(cout, generator=g) - 0.5).to(gpu_device)
    wp = engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 32 if cout <= 32 else 64)
    outs = []
    try:
        for L in (lib, ablation_lib):
            if L is ablation_lib:
                L.esr_x3_set_tile_map(0)
            out = torch.zeros(B, H + 2, W + 2, cout, device=gpu_device)
            o = engine._conv_out(out, cout, 0, H, W, True)
            _lib.check(L.esr_conv3x3_fwd(x.data_ptr(), B, H, W, cp, cin, wp.data_ptr(), bd.data_ptr(), cout,
                                         ctypes.byref(o), _stream()), 'conv')
            torch.cuda.synchronize()
            outs.append(out)
    finally:
        ablation_lib.esr_x3_set_tile_map(1)
    assert torch.equal(outs[0], outs[1])
    ref = F.leaky_relu(F.conv2d(_nchw(x, 0, cin), w.double(), bd.cpu().double(), padding=1), 0.2)
    assert normwise_rel(_nchw(outs[0], 0, cout), ref) < 1e-5


def test_conv3x3_planar_output(gpu_device):
    lib = _lib.load()
    B, H, W, cin = 2, 19, 45, 72
    x = _padded(B, H, W, cin, cin, gpu_device, 4)
    w = torch.randn(3, cin, 3, 3, generator=torch.Generator().manual_seed(5)) * 0.05
    b = torch.tensor([0.1, -0.2, 0.3])
    wp = engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 32)
    out = torch.full((B, 3, H, W), 7.0, device=gpu_device)
    o = engine._conv_out(out, 0, 0, H, W, False, planar=1)
    _lib.check(lib.esr_conv3x3_fwd(x.data_ptr(), B, H, W, cin, cin, wp.data_ptr(), b.to(gpu_device).data_ptr(), 3,
                                   ctypes.byref(o), _stream()), 'conv')
    torch.cuda.synchronize()
    ref = F.conv2d(_nchw(x, 0, cin), w.double(), b.double(), padding=1)
    assert normwise_rel(out.cpu(), ref) < 1e-5


@pytest.mark.parametrize('H,W', [(6, 9), (16, 40)])
def test_upconv2x_phases(gpu_device, H, W):
    lib = _lib.load()
    B = 2
    x = _padded(B, H, W, 64, 64, gpu_device, 6)
    w = torch.randn(64, 64, 3, 3, generator=torch.Generator().manual_seed(7)) * 0.05
    b = torch.randn(64, generator=torch.Generator().manual_seed(8)) * 0.1
    out = torch.zeros(B, 2 * H + 2, 2 * W + 2, 64, device=gpu_device)
    bd = b.to(gpu_device)
    for py in (0, 1):
        for px in (0, 1):
            wp = engine.pack_conv_weight(engine.fold_upconv_phase(w.to(gpu_device), py, px), list(range(64)), 64)
            o = engine._conv_out(out, 64, 0, 2 * H, 2 * W, True, sy=2, sx=2, oy=py, ox=px)
            _lib.check(lib.esr_upconv2x_phase_fwd(x.data_ptr(), B, H, W, 64, 64, wp.data_ptr(), bd.data_ptr(), 64,
                                                  py, px, ctypes.byref(o), _stream()), 'upconv')
    torch.cuda.synchronize()
    ref = F.leaky_relu(F.conv2d(F.interpolate(_nchw(x, 0, 64), scale_factor=2, mode='nearest'), w.double(),
                                b.double(), padding=1), 0.2)
    assert normwise_rel(_nchw(out, 0, 64), ref) < 1e-5


@pytest.mark.parametrize('name', ['cem_bicubic', 'cem_learned13'])
def test_cem_filter_ops_vs_golden(gpu_device, name):
    d = golden(name)
    cem = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=d['input_kernel'] if 'input_kernel' in d else None)
    m = cem.WrapArchitecture_PyTorch(torch.nn.Identity()).to(gpu_device)
    with torch.no_grad():
        down = m.DownscaleOP(torch.from_numpy(d['down_hr']).to(gpu_device))
    assert normwise_rel(down.cpu(), d['down_out']) < 1e-5
    design = O.cem_design(4, d['input_kernel'] if 'input_kernel' in d else None)
    v = torch.rand(2, 3, 11, 14, generator=torch.Generator().manual_seed(9))
    with torch.no_grad():
        inv = m.Conv_LR_with_Inv_hTh_OP(v.to(gpu_device)).cpu()
        up = m.Upscale_OP(v.to(gpu_device)).cpu()
    assert normwise_rel(inv, O.cem_inv(v, design['inv_hTh'])) < 1e-5
    assert normwise_rel(up, O.cem_upscale(v, design['ds_kernel'])) < 1e-5


@pytest.mark.parametrize('name', ['cem_bicubic', 'cem_learned13'])
@pytest.mark.parametrize('mode', ['train', 'eval'])
def test_cem_step_vs_golden(gpu_device, name, mode):
    """CEM back-projection alone: a fixed generator output through engine.cem_apply."""
    d = golden(name)
    cem = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=d['input_kernel'] if 'input_kernel' in d else None)
    m = cem.WrapArchitecture_PyTorch(torch.nn.Identity()).to(gpu_device)
    gen = torch.from_numpy(d['fwd_%s_gen' % mode]).to(gpu_device)
    lr = torch.from_numpy(d['fwd_%s_lr' % mode])
    mL = int(cem.invalidity_margins_LR) if mode == 'eval' else 0
    lr = F.pad(lr, (mL,) * 4, mode='replicate').to(gpu_device).contiguous()
    B, _, H, W = lr.shape
    out = engine.cem_apply(_lib.load(), m, gen, lr, B, H, W, 4 * mL, _stream())
    torch.cuda.synchronize()
    assert normwise_rel(out.cpu(), d['fwd_%s_out' % mode]) < 1e-5


def _product_model(d, dev, precision):
    keys, params = fixture_params(d)
    latent = bool(int(d['latent']))
    sf = fixture_upscale(d)
    net = esr_amd.RRDBNet(3, 3, 64, int(d['nb']), upscale=sf,
                          latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    mode = str(d['cem_mode'])
    model = net
    if mode != 'none':
        cem = C.CEMnet(C.Get_CEM_Config(sf), upscale_kernel=d['kernel'] if 'kernel' in d else None)
        model = cem.WrapArchitecture_PyTorch(net)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    assert not unexpected and all('Filter' in k for k in missing)
    model.to(dev)
    model.train(mode == 'train')
    engine.set_precision(model, precision)
    return model


@pytest.mark.parametrize('precision', ['f32', 'x3'])
@pytest.mark.parametrize('name', golden_names('rrdb_'))
def test_generator_vs_reference_golden(gpu_device, name, precision):
    d = golden(name)
    model = _product_model(d, gpu_device, precision)
    with torch.no_grad():
        out = model(fixture_input(d).to(gpu_device))
    torch.cuda.synchronize()
    assert out.shape == d['out'].shape
    assert normwise_rel(out.cpu(), d['out']) < 1e-4


def _big_model(nb, latent, dev, precision, seed=21, w_scale=0.5):
    from oracle.recipe import seeded_params
    net = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], seed, w_scale=w_scale)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    engine.set_precision(model, precision)
    return model.to(dev), params


@pytest.mark.parametrize('precision', ['f32', 'x3'])
@pytest.mark.parametrize('latent', [False, True])
def test_full_size_rrdb23_cem_vs_oracle(gpu_device, latent, precision):
    """C1 shape (128² LR -> 512², RRDB-23 + CEM eval pre-pad) against the CPU oracle: the north_star 1e-3 bar."""
    model, params = _big_model(23, latent, gpu_device, precision)
    model.eval()
    from oracle.recipe import seeded_inputs
    lr, z = seeded_inputs(22, (1, 3, 128, 128), (1, 3, 512, 512) if latent else None)
    x = torch.from_numpy(lr)
    if latent:
        x = torch.cat([torch.from_numpy(z).reshape(1, 48, 128, 128), x], 1)
    with torch.no_grad():
        out = model(x.to(gpu_device)).cpu()
        design = O.cem_design(4)
        ref = O.sr_forward(x, O.strip_prefix(params), 23, latent, design, pre_pad=True)
    err = normwise_rel(out, ref)
    mse = float(((out.double() - ref.double()) ** 2).mean())
    print('full-size normwise rel err (latent=%s, %s): %.3e, PSNR vs ref %.1f dB'
          % (latent, precision, err, 10 * np.log10(1 / max(mse, 1e-30))))
    assert err < 1e-3
    assert mse < 1e-8


@pytest.mark.parametrize('latent', [False, True])
@pytest.mark.parametrize('B,h,w', [(2, 9, 13), (3, 16, 5)])
def test_hr_convs_fused_equals_unfused(gpu_device, monkeypatch, latent, B, h, w):
    """x3 inference runs HR_conv0 + HR_conv1 as esr_hr_convs_x3 + esr_hr1_sum (HR_conv0's activations never stored;
    HR_conv1's 27 per-tap partial products from HR_conv0's epilogue, summed over each pixel's 3×3 neighbours): equal to
    the two convs as the training forward launches them (HR_conv1 on the narrow-N kernel) up to the summation order,
    and on the float64 oracle.  Ragged widths (tiles past the image edge), the latent slot, the CEM pre-pad."""
    model, params = _big_model(1, latent, gpu_device, 'x3', seed=41)
    model.eval()
    g = torch.Generator().manual_seed(42)
    x = torch.rand(B, 3, h, w, generator=g)
    if latent:
        z = 2 * torch.rand(B, 3, 4 * h, 4 * w, generator=g) - 1
        x = torch.cat([z.reshape(B, 48, h, w), x], 1)
    xd = x.to(gpu_device)
    outs = {}
    for fuse in (True, False):
        monkeypatch.setattr(engine, 'FUSE_HR1', fuse)
        with torch.no_grad():
            outs[fuse] = model(xd).cpu()
    err = normwise_rel(outs[True], outs[False])
    ref = O.sr_forward(x, O.strip_prefix(params), 1, latent, O.cem_design(4), pre_pad=True)
    err_ref = normwise_rel(outs[True], ref)
    print('fused vs unfused %.2e, fused vs float64 oracle %.2e, unfused vs oracle %.2e'
          % (err, err_ref, normwise_rel(outs[False], ref)))
    assert err < 2e-6
    assert err_ref < 1e-5


@pytest.mark.parametrize('precision', ['x3', 'f32'])
@pytest.mark.parametrize('latent', [False, True])
def test_c2_production_grid_vs_oracle_and_batch1(gpu_device, latent, precision):
    """Config 2 at its real grid: B=32 × 128² LR, RRDB-23 + CEM eval (pre-pad → 148² tall batch image, the production
    tile count and XCD remainder split of every conv launch).  Two images of the batch (first and last: different
    tiles of the tall image, the last one touching its bottom edge) against the CPU oracle at the north_star 1e-3 bar,
    and bitwise equal to the same images run alone (B=1)."""
    B = 32
    model, params = _big_model(23, latent, gpu_device, precision, seed=23)
    model.eval()
    g = torch.Generator().manual_seed(24)
    lr = torch.rand(B, 3, 128, 128, generator=g)
    x = lr
    if latent:  # per-image constant Z as in training, a different one per image
        z = (2 * torch.rand(B, 3, 1, 1, generator=g) - 1).expand(B, 3, 512, 512).contiguous()
        x = torch.cat([z.view(B, 48, 128, 128), lr], 1)
    xd = x.to(gpu_device)
    with torch.no_grad():
        out = model(xd)
        torch.cuda.synchronize()
        design = O.cem_design(4)
        for i in (0, B - 1):
            alone = model(xd[i:i + 1].contiguous())
            assert torch.equal(out[i:i + 1], alone), i
            ref = O.sr_forward(x[i:i + 1], O.strip_prefix(params), 23, latent, design, pre_pad=True)
            err = normwise_rel(out[i:i + 1].cpu(), ref)
            print('C2 grid image %d (latent=%s, %s): normwise %.3e' % (i, latent, precision, err))
            assert err < 1e-3
    assert tuple(out.shape) == (B, 3, 512, 512)


@pytest.mark.parametrize('precision', ['f32', 'x3'])
def test_cem_consistency_and_batch_invariance(gpu_device, precision):
    """Size-independent properties at a larger batch: (1) CEM consistency — DownscaleOP(SR) reproduces the LR input in
    the valid interior (the module's defining property, CEMnet.py:186-189); (2) every image of a batch equals the same
    image run alone, bitwise; (3) two runs are bitwise identical."""
    model, _ = _big_model(2, False, gpu_device, precision, seed=31)
    model.train(False)
    x = torch.rand(4, 3, 64, 80, generator=torch.Generator().manual_seed(32)).to(gpu_device)
    with torch.no_grad():
        y = model(x)
        y2 = model(x)
        y1 = model(x[2:3].contiguous())
        lr_back = model.DownscaleOP(y)
    assert torch.equal(y, y2)
    assert torch.equal(y[2:3], y1)
    m = 12  # stay clear of the CEM invalidity margin (10 LR px for the bicubic kernel)
    err = (lr_back - x)[:, :, m:-m, m:-m].abs().max().item()
    assert err < 1e-4, err


@pytest.mark.parametrize('img_scale', [1.0, 1e-3])
def test_x3_trained_scale_weights_and_small_activations(gpu_device, img_scale):
    """x3 accuracy away from the fixtures' weight scales: define_G's training-time init (kaiming × 0.1,
    networks.py:97-98, the scale trained ESRGAN weights keep) with small biases, on images in [0, 1] and in [0, 1e-3].
    At 1e-3 most activations sit below 2^-3, where the f16 lo part of a split value is subnormal (absolute step 2^-24):
    the product keeps ~2^-24 absolute instead of 2^-22 relative accuracy.  The x3 output stays within 1e-4 normwise of
    the float64 oracle (the north_star bar is 1e-3), next to the exact-fp32 path's own error."""
    torch.manual_seed(51)
    net = esr_amd.RRDBNet(3, 3, 64, 2, num_latent_channels=0)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net)
    esr_amd.init_weights(model, 'kaiming', scale=0.1)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith('bias'):
                p.uniform_(-0.01 * img_scale, 0.01 * img_scale)
    params = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    model.eval().to(gpu_device)
    x = torch.rand(2, 3, 40, 52, generator=torch.Generator().manual_seed(52)) * img_scale
    errs = {}
    with torch.no_grad():
        ref = O.sr_forward(x.double(), {k: v.double() for k, v in O.strip_prefix(
            {k: v for k, v in params.items() if 'Filter' not in k}).items()}, 2, False, O.cem_design(4), pre_pad=True)
        for prec in ('f32', 'x3'):
            engine.set_precision(model, prec)
            errs[prec] = normwise_rel(model(x.to(gpu_device)).cpu(), ref)
    print('image scale %g: normwise vs float64 oracle  f32 %.2e  x3 %.2e' % (img_scale, errs['f32'], errs['x3']))
    assert errs['f32'] < 1e-5
    assert errs['x3'] < 1e-4


@pytest.mark.parametrize('precision', ['x3', 'f32'])
def test_multistream_forward_bitwise_equals_one_stream(gpu_device, monkeypatch, precision):
    """engine._multistream_forward (the batch in S parts on S HIP streams, config 2's default) at a small shape with
    the part-size gate lifted: S = 2 and 3 (ragged parts: 9 images) bitwise equal to one stream, latent slot and CEM
    pre-pad included; the output is stream-ordered for the caller (read on the current stream right after)."""
    model, _ = _big_model(1, True, gpu_device, precision, seed=61)
    model.eval()
    g = torch.Generator().manual_seed(62)
    B, h, w = 9, 12, 20
    z = 2 * torch.rand(B, 3, 1, 1, generator=g) - 1
    x = torch.cat([z.expand(B, 3, 4 * h, 4 * w).reshape(B, 48, h, w), torch.rand(B, 3, h, w, generator=g)], 1)
    xd = x.to(gpu_device)
    monkeypatch.setattr(engine, 'STREAM_MIN_PART_PIXELS', 0)
    outs = {}
    with torch.no_grad():
        for s in (1, 2, 3):
            monkeypatch.setattr(engine, 'STREAMS', s)
            assert engine.use_streams(xd.shape, model) == (s > 1)
            outs[s] = model(xd).cpu()
    assert torch.equal(outs[1], outs[2])
    assert torch.equal(outs[1], outs[3])


def test_multistream_overflow_in_one_part_reruns_the_batch(gpu_device, monkeypatch):
    """An f16-range overflow in the second of two stream parts: the whole batch reruns in exact fp32."""
    model, _ = _big_model(1, False, gpu_device, 'x3', seed=41, w_scale=1.0)
    model.eval()
    monkeypatch.setattr(engine, 'STREAM_MIN_PART_PIXELS', 0)
    monkeypatch.setattr(engine, 'STREAMS', 2)
    x = torch.rand(8, 3, 16, 16, generator=torch.Generator().manual_seed(43))
    x[5:] *= 3.0e5  # the second part's inputs drive conv_first beyond 65504
    xd = x.to(gpu_device)
    before = engine.OVERFLOW_RERUNS
    with torch.no_grad():
        y = model(xd)
        engine.set_precision(model, 'f32')
        ref = model(xd)
    assert engine.OVERFLOW_RERUNS == before + 1
    assert torch.equal(y, ref)


def test_x3_overflow_falls_back_to_exact_f32(gpu_device):
    """Activations beyond the f16 range must not corrupt the x3 path: the overflow flag triggers an exact-fp32 rerun."""
    model, _ = _big_model(1, False, gpu_device, 'x3', seed=41, w_scale=1.0)
    with torch.no_grad():
        model.generated_image_model.model[0].weight.mul_(2.0e5)  # conv_first output far beyond 65504
    model.eval()
    x = torch.rand(1, 3, 16, 16, generator=torch.Generator().manual_seed(42)).to(gpu_device)
    before = engine.OVERFLOW_RERUNS
    with torch.no_grad():
        y = model(x)
        engine.set_precision(model, 'f32')
        ref = model(x)
    assert engine.OVERFLOW_RERUNS == before + 1
    assert torch.equal(y, ref)


@pytest.mark.parametrize('cin,cout,H,W', [(8, 64, 5, 7), (72, 32, 13, 37), (200, 64, 9, 33), (64, 32, 17, 31),
                                          (136, 32, 8, 32), (16, 64, 1, 1), (104, 32, 33, 70)])
def test_conv3x3_layer_x3(gpu_device, cin, cout, H, W):
    lib = _lib.load()
    B = 2
    cp = cin + 8
    xf = _padded(B, H, W, cp, cin, gpu_device, 11)
    xf[..., cin:] = 0
    g = torch.Generator().manual_seed(12)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.1
    b = torch.rand(cout, generator=g) - 0.5
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 32 if cout <= 32 else 64))
    res = _padded(B, H, W, 80, 80, gpu_device, 13)
    out = torch.zeros(B, H + 2, W + 2, 80, device=gpu_device)
    out2 = torch.zeros(B, H + 2, W + 2, 64, device=gpu_device)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    xs, rs = engine.to_split(xf), engine.to_split(res)
    o = engine._conv_out(out, 80, 8, H, W, True, r1=rs, r1_cp=80, r1_coff=0, s1=0.2, r2=rs, r2_cp=80, r2_coff=8,
                         s2=0.5, out2=out2, out2_cp=64, out2_coff=0)
    _lib.check(lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.to(gpu_device).data_ptr(),
                                      scale, cout, ctypes.byref(o), ovf.data_ptr(), _stream()), 'conv_x3')
    torch.cuda.synchronize()
    got = engine.from_split(out)
    ref = F.leaky_relu(F.conv2d(_nchw(engine.from_split(xs), 0, cin), w.double(), b.double(), padding=1), 0.2)
    rsv = engine.from_split(rs)
    ref = 0.5 * (0.2 * ref + _nchw(rsv, 0, cout)) + _nchw(rsv, 8, 8 + cout)
    err = normwise_rel(_nchw(got, 8, 8 + cout), ref)
    assert err < 1e-5, err
    assert torch.equal(out2[:, 1:-1, 1:-1, :cout], out[:, 1:-1, 1:-1, 8:8 + cout])
    assert torch.all(out[..., :8] == 0) and torch.all(out[..., 8 + cout:] == 0)
    assert torch.all(out[:, 0] == 0) and torch.all(out[:, -1] == 0) and torch.all(out[:, :, 0] == 0)
    assert int(ovf.item()) == 0


@pytest.mark.parametrize('cin,cout,B,H,W', [(64, 32, 3, 40, 148), (136, 32, 5, 17, 45), (104, 24, 2, 33, 70),
                                            (16, 32, 1, 1, 1), (160, 32, 4, 96, 33)])
def test_x3_ring_kernel_bitwise_equals_classic(gpu_device, ablation_lib, cin, cout, B, H, W):
    """The N<=32 ring kernels (two tiles per workgroup, 3-deep LDS-DMA ring, counted vmcnt; and the persistent variant
    that streams several tile pairs per workgroup with a per-wave epilogue) run the classic kernel's MFMA sequence per
    accumulator: outputs, residual epilogue and out2 must agree bit for bit, including odd tile counts (the second tile
    of the last pair is beyond the batch) and partial column tiles (W = 148 and 1: a 4- and a 1-column last tile of the
    default 12-column kernel)."""
    lib = _lib.load()
    cp = cin + 8
    xs = engine.to_split(_padded(B, H, W, cp, cin, gpu_device, 21))
    g = torch.Generator().manual_seed(22)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.1
    b = (torch.rand(cout, generator=g) - 0.5).to(gpu_device)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 32))
    rs = engine.to_split(_padded(B, H, W, 40, 40, gpu_device, 23))
    outs = []
    try:
        # classic one-stage (default), ring always, persistent ring always, ring / classic with the compiler-scheduled
        # fragment reads, two-stage classic with prefetch 1 / 2, the round-1 automatic choice, the column-tile kernel
        # (16-column tiles, LDS / register weights; 12-column tiles at three workgroups per CU, the default where column
        # tiles pay) (none may change a bit)
        # (the product library's automatic choice first, then the ablation library's variants)
        for variant in (0, 2, 17, 18, 20, 21, 22, 25, 26, 27, 28, 24, 50, 60, 61, 62, 64):
            L = lib if variant == 0 else ablation_lib
            if L is ablation_lib:
                L.esr_x3_set_kernel(variant)
            out = torch.zeros(B, H + 2, W + 2, 40, device=gpu_device)
            out2 = torch.zeros(B, H + 2, W + 2, 32, device=gpu_device)
            o = engine._conv_out(out, 40, 8, H, W, True, r1=rs, r1_cp=40, r1_coff=0, s1=0.2, out2=out2, out2_cp=32,
                                 out2_coff=0)
            _lib.check(L.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                            cout, ctypes.byref(o), None, _stream()), 'conv_x3')
            torch.cuda.synchronize()
            outs.append((out, out2))
    finally:
        ablation_lib.esr_x3_set_kernel(1)
    for k in range(1, len(outs)):
        assert torch.equal(outs[0][0], outs[k][0]) and torch.equal(outs[0][1], outs[k][1]), k
    ref = F.leaky_relu(F.conv2d(_nchw(engine.from_split(xs), 0, cin), w.double(), b.cpu().double(), padding=1), 0.2)
    ref = 0.2 * ref + _nchw(engine.from_split(rs), 0, cout)
    assert normwise_rel(_nchw(engine.from_split(outs[1][0]), 8, 8 + cout), ref) < 1e-5


@pytest.mark.parametrize('cin,B,H,W', [(192, 3, 21, 70), (72, 1, 5, 9), (192, 3, 21, 76), (64, 2, 9, 4)])
def test_x3_n64_explicit_reads_bitwise(gpu_device, ablation_lib, cin, B, H, W):
    """The N = 64 classic kernel with explicit counted-wait fragment reads (default) against the same kernel with the
    compiler-scheduled reads (esr_x3_set_kernel 20): same MFMA order per accumulator, so bit for bit.  W = 76 and 4
    end in a 4-column partial tile of the default 12-column kernel."""
    lib = _lib.load()
    cp = cin + 8
    xs = engine.to_split(_padded(B, H, W, cp, cin, gpu_device, 31))
    g = torch.Generator().manual_seed(32)
    w = torch.randn(64, cin, 3, 3, generator=g) * 0.05
    b = (torch.rand(64, generator=g) - 0.5).to(gpu_device)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 64))
    outs = []
    try:
        # default (column tiles), compiler-scheduled reads, 8-row tiles at two workgroups per CU, the round-1 default,
        # column tiles with register weights
        for variant in (1, 20, 23, 24, 60):
            L = lib if variant == 1 else ablation_lib
            if L is ablation_lib:
                L.esr_x3_set_kernel(variant)
            out = torch.zeros(B, H + 2, W + 2, 64, device=gpu_device)
            o = engine._conv_out(out, 64, 0, H, W, True)
            _lib.check(L.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                            64, ctypes.byref(o), None, _stream()), 'conv_x3')
            torch.cuda.synchronize()
            outs.append(out)
    finally:
        ablation_lib.esr_x3_set_kernel(1)
    for k in range(1, len(outs)):
        assert torch.equal(outs[0], outs[k]), k
    assert outs[0].abs().sum() > 0


@pytest.mark.parametrize('cout,cin,B,H,W', [(32, 72, 3, 21, 70), (64, 96, 2, 37, 150), (32, 64, 5, 33, 40)])
def test_x3_xcd_tile_map_bitwise(gpu_device, ablation_lib, cout, cin, B, H, W):
    """XCD-grouped block -> tile order (default, esr_x3_set_tile_map 1) against row-major blockIdx order (0): a
    renumbering of the same tiles, so bit for bit; grids of 15 / 30 / 45 (16-row) and 8-row tiles are not multiples of
    the 8 XCDs, which exercises the remainder split of xcd_tile."""
    lib = _lib.load()
    cp = cin + 8
    xs = engine.to_split(_padded(B, H, W, cp, cin, gpu_device, 41))
    g = torch.Generator().manual_seed(42)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    b = (torch.rand(cout, generator=g) - 0.5).to(gpu_device)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), cout))
    outs = []
    try:
        for L in (lib, ablation_lib):
            if L is ablation_lib:
                L.esr_x3_set_tile_map(0)
            out = torch.zeros(B, H + 2, W + 2, cout, device=gpu_device)
            o = engine._conv_out(out, cout, 0, H, W, True)
            _lib.check(L.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                            cout, ctypes.byref(o), None, _stream()), 'conv_x3')
            torch.cuda.synchronize()
            outs.append(out)
    finally:
        ablation_lib.esr_x3_set_tile_map(1)
    assert torch.equal(outs[0], outs[1])
    ref = F.leaky_relu(F.conv2d(_nchw(engine.from_split(xs), 0, cin), w.double(), b.cpu().double(), padding=1), 0.2)
    assert normwise_rel(_nchw(engine.from_split(outs[0]), 0, cout), ref) < 1e-5


@pytest.mark.parametrize('cin,cout,B,H,W', [(192, 64, 2, 24, 40), (72, 40, 1, 9, 21)])
def test_x3_nsplit_bitwise(gpu_device, ablation_lib, cin, cout, B, H, W):
    """An N = 64 conv on a small grid in the product's choice (12-column N = 64 tiles, two per CU) against the same
    conv as two N = 32 launches over the halves of its packed weights (round 3's N split, esr_x3_set_nsplit) and in
    16-column tiles (variant 50): the RDB conv5 epilogue (LeakyReLU off, 0.2 x conv + residual at a channel offset, a
    dual output at another offset) must land in the same channels, bit for bit."""
    lib = _lib.load()
    cp = cin + 8
    xs = engine.to_split(_padded(B, H, W, cp, cin, gpu_device, 51))
    rs = engine.to_split(_padded(B, H, W, cp, cp, gpu_device, 52))
    g = torch.Generator().manual_seed(53)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    b = (torch.rand(cout, generator=g) - 0.5).to(gpu_device)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 64))
    outs = []
    try:
        for L, nsplit, variant in ((lib, None, None), (ablation_lib, 1, 1), (ablation_lib, 0, 50)):
            if L is ablation_lib:
                L.esr_x3_set_nsplit(nsplit)
                L.esr_x3_set_kernel(variant)
            out = torch.zeros(B, H + 2, W + 2, 80, device=gpu_device)
            out2 = torch.zeros(B, H + 2, W + 2, 88, device=gpu_device)
            o = engine._conv_out(out, 80, 8, H, W, False, r1=rs, r1_cp=cp, r1_coff=16, s1=0.2, out2=out2, out2_cp=88,
                                 out2_coff=24)
            _lib.check(L.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                            cout, ctypes.byref(o), None, _stream()), 'conv_x3')
            torch.cuda.synchronize()
            outs.append((out, out2))
    finally:
        ablation_lib.esr_x3_set_nsplit(0)
        ablation_lib.esr_x3_set_kernel(1)
    for k in (1, 2):
        assert torch.equal(outs[0][0], outs[k][0]) and torch.equal(outs[0][1], outs[k][1]), k
    ref = F.conv2d(_nchw(engine.from_split(xs), 0, cin), w.double(), b.cpu().double(), padding=1)
    assert normwise_rel(_nchw(engine.from_split(outs[0][0]), 8, 8 + cout), ref * 0.2 +
                        _nchw(engine.from_split(rs), 16, 16 + cout)) < 1e-5


# default, direct register epilogue 16- / 8-row, classic, column tiles
@pytest.mark.parametrize('variant', [1, 27, 28, 24, 50, 64])
def test_conv3x3_x3_planar_output(gpu_device, variant, request):
    lib = _lib.load() if variant == 1 else request.getfixturevalue('ablation_lib')
    B, H, W, cin = 2, 19, 45, 72
    x = engine.to_split(_padded(B, H, W, cin, cin, gpu_device, 14))
    w = torch.randn(3, cin, 3, 3, generator=torch.Generator().manual_seed(15)) * 0.05
    b = torch.tensor([0.1, -0.2, 0.3])
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 32))
    out = torch.full((B, 3, H, W), 7.0, device=gpu_device)
    o = engine._conv_out(out, 0, 0, H, W, False, planar=1)
    try:
        if variant != 1:
            lib.esr_x3_set_kernel(variant)
        _lib.check(lib.esr_conv3x3_fwd_x3(x.data_ptr(), B, H, W, cin, cin, wx.data_ptr(),
                                          b.to(gpu_device).data_ptr(), scale, 3, ctypes.byref(o), None, _stream()),
                   'conv_x3')
        torch.cuda.synchronize()
    finally:
        if variant != 1:
            lib.esr_x3_set_kernel(1)
    ref = F.conv2d(_nchw(engine.from_split(x), 0, cin), w.double(), b.double(), padding=1)
    assert normwise_rel(out.cpu(), ref) < 1e-5


@pytest.mark.parametrize('variant', [1, 24])  # column-tile kernel (default), classic kernel
@pytest.mark.parametrize('H,W', [(6, 9), (16, 40), (37, 21), (5, 36), (3, 4)])  # 36, 4: a 4-column last tile
def test_upconv2x_phases_x3(gpu_device, H, W, variant, request):
    lib = _lib.load() if variant == 1 else request.getfixturevalue('ablation_lib')
    if variant != 1:
        lib.esr_x3_set_kernel(variant)
    B = 2
    x = engine.to_split(_padded(B, H, W, 64, 64, gpu_device, 16))
    w = torch.randn(64, 64, 3, 3, generator=torch.Generator().manual_seed(17)) * 0.05
    b = torch.randn(64, generator=torch.Generator().manual_seed(18)) * 0.1
    out = torch.zeros(B, 2 * H + 2, 2 * W + 2, 64, device=gpu_device)
    bd = b.to(gpu_device)
    for py in (0, 1):
        for px in (0, 1):
            wx, scale = engine.pack_x3(engine.pack_conv_weight(engine.fold_upconv_phase(w.to(gpu_device), py, px),
                                                               list(range(64)), 64))
            o = engine._conv_out(out, 64, 0, 2 * H, 2 * W, True, sy=2, sx=2, oy=py, ox=px)
            _lib.check(lib.esr_upconv2x_phase_fwd_x3(x.data_ptr(), B, H, W, 64, 64, wx.data_ptr(), bd.data_ptr(),
                                                     scale, 64, py, px, ctypes.byref(o), None, _stream()), 'up_x3')
    torch.cuda.synchronize()
    if variant != 1:
        lib.esr_x3_set_kernel(1)
    ref = F.leaky_relu(F.conv2d(F.interpolate(_nchw(engine.from_split(x), 0, 64), scale_factor=2, mode='nearest'),
                                w.double(), b.double(), padding=1), 0.2)
    assert normwise_rel(_nchw(engine.from_split(out), 0, 64), ref) < 1e-5


@pytest.mark.parametrize('B,H,W,ki,kd,M', [(32, 148, 148, 27, 17, 40), (2, 21, 37, 13, 13, 0), (1, 9, 70, 33, 25, 8)])
def test_cem_tiled_stencils_bitwise_equal_direct(gpu_device, ablation_lib, B, H, W, ki, kd, M):
    """The LDS-tiled inverse-filter and up-add kernels (default) against the direct kernels (esr_cem_set_direct(1)):
    same taps in the same order per output, so bit for bit — at the config-2 shape (B=32, 148² LR) and at ragged
    shapes (tiles past the image edge, windows clamped on every side) — and against float64.  The register-window down
    kernel (default at sf 4, kd 17) against the LDS-tiled one (direct mode) within rounding, and against float64."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(61)
    r = torch.randn(B, 3, H, W, generator=g).to(gpu_device)
    wi = (torch.randn(ki, ki, generator=g) * 0.05).to(gpu_device)
    wu = (torch.randn(kd, kd, generator=g) * 0.1).to(gpu_device)
    gen = torch.randn(B, 3, 4 * H, 4 * W, generator=g).to(gpu_device)
    lr = torch.randn(B, 3, H, W, generator=g).to(gpu_device)
    res, downs = {}, {}
    try:
        for direct in (1, 0):
            L = ablation_lib if direct else lib  # the direct kernels: ablation library only
            if direct:
                L.esr_cem_set_direct(1)
            downs[direct] = []
            for ph in (1, 2):
                d = torch.full((B, 3, H, W), 7.0, device=gpu_device)
                _lib.check(L.esr_cem_down(gen.data_ptr(), lr.data_ptr(), d.data_ptr(), B, H, W, 4, ph, wu.data_ptr(),
                                            kd, 0, _stream()), 'down')
                downs[direct].append(d)
            q = torch.empty_like(r)
            _lib.check(L.esr_cem_inv(r.data_ptr(), q.data_ptr(), B, H, W, wi.data_ptr(), ki, _stream()), 'inv')
            outs = []
            for ph in (1, 2):
                out = torch.full((B, 3, 4 * H - 2 * M, 4 * W - 2 * M), 7.0, device=gpu_device)
                _lib.check(L.esr_cem_up_add(q.data_ptr(), gen.data_ptr(), out.data_ptr(), B, H, W, 4, ph,
                                              wu.data_ptr(), kd, M, _stream()), 'up_add')
                outs.append(out)
            torch.cuda.synchronize()
            res[direct] = (q, outs)
    finally:
        ablation_lib.esr_cem_set_direct(0)
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)
    for a, b in zip(downs[0], downs[1]):  # FMA contraction differs between the two down kernels: rounding-level
        assert normwise_rel(a.cpu().double(), b.cpu().double()) < 1e-6
    gd = F.conv2d(F.pad(gen.double().cpu().view(B * 3, 1, 4 * H, 4 * W), (kd // 2,) * 4, mode='replicate'),
                  wu.double().cpu().view(1, 1, kd, kd))
    for ph, got in zip((1, 2), downs[0]):
        ref = lr.double().cpu().view(B * 3, 1, H, W) - gd[:, :, ph::4, ph::4]
        assert normwise_rel(got.cpu().view_as(ref), ref) < 1e-5
    # float64: replicate-padded cross-correlation (inverse filter); zero-stuffed ×4 grid at phase ph, replicate-padded
    rd = r.double().cpu()
    ref_q = F.conv2d(F.pad(rd.view(B * 3, 1, H, W), (ki // 2,) * 4, mode='replicate'), wi.double().cpu().view(1, 1, ki, ki))
    assert normwise_rel(res[0][0].cpu().view(B * 3, 1, H, W), ref_q) < 1e-5
    qd = res[0][0].double().cpu().view(B * 3, 1, H, W)
    for ph, got in zip((1, 2), res[0][1]):
        st = torch.zeros(B * 3, 1, 4 * H, 4 * W, dtype=torch.float64)
        st[:, :, ph::4, ph::4] = qd
        up = F.conv2d(F.pad(st, (kd // 2,) * 4, mode='replicate'), wu.double().cpu().view(1, 1, kd, kd))
        ref = gen.double().cpu().view(B * 3, 1, 4 * H, 4 * W) + up
        ref = ref[:, :, M:4 * H - M, M:4 * W - M]
        assert normwise_rel(got.cpu().view_as(ref), ref) < 1e-5


@pytest.mark.parametrize('cin,B,H,W', [(64, 2, 19, 45), (72, 3, 17, 61), (64, 1, 1, 1), (72, 2, 40, 30),
                                       (64, 4, 33, 92)])
def test_conv3x3_x3_narrow_planar(gpu_device, ablation_lib, cin, B, H, W):
    """The narrow-N x3 path (cout 3, planar fp32 output: HR_conv1 -> CEM; taps in the MFMA M dimension, shifted
    partial products summed from LDS) against float64, and against the N = 32 tile path it replaces (same x3 products,
    another tap summation order), over odd sizes, partial 30-column tiles, the latent 72-channel input (a half-filled
    last K chunk whose channels past cin are never read) and tiles straddling images of the tall batch image."""
    lib = _lib.load()
    cp = cin
    xs = engine.to_split(_padded(B, H, W, cp, cin, gpu_device, 31))
    g = torch.Generator().manual_seed(32)
    w = torch.randn(3, cin, 3, 3, generator=g) * 0.05
    b = (torch.rand(3, generator=g) - 0.5).to(gpu_device)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w.to(gpu_device), list(range(cin)), 32))
    outs = []
    try:
        for L in (lib, ablation_lib):  # narrow-N (product) / N = 32 tiles (ablation library)
            if L is ablation_lib:
                L.esr_x3_set_narrow(0)
            out = torch.full((B, 3, H, W), 7.0, device=gpu_device)
            o = engine._conv_out(out, 0, 0, H, W, False, planar=1)
            _lib.check(L.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale, 3,
                                            ctypes.byref(o), None, _stream()), 'conv_x3')
            torch.cuda.synchronize()
            outs.append(out.cpu())
    finally:
        ablation_lib.esr_x3_set_narrow(1)
    ref = F.conv2d(_nchw(engine.from_split(xs), 0, cin), w.double(), b.cpu().double(), padding=1)
    for out in outs:
        assert normwise_rel(out, ref) < 2e-6, normwise_rel(out, ref)
    assert float((outs[0].double() - outs[1].double()).abs().max() / ref.abs().max()) < 2e-6
