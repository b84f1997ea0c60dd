"""Host-side logic of the product package, CPU only: CEM filter design vs golden, module/state_dict layout vs the
reference, weight packing / upconv folding algebra, C-ABI library exports, and loud failure without a GPU."""
import ctypes
import json
import math
import os
import re
import subprocess

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import fixture_upscale, REPO, golden, golden_names

import esr_amd
from esr_amd import CEMnet as C
from esr_amd import engine
from esr_amd import _lib


@pytest.mark.parametrize('name', ['cem_bicubic', 'cem_learned13'])
def test_product_cem_design_exact(name):
    d = golden(name)
    cem = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=d['input_kernel'] if 'input_kernel' in d else None)
    np.testing.assert_array_equal(cem.ds_kernel, d['ds_kernel'])
    np.testing.assert_array_equal(cem.inv_hTh, d['inv_hTh'])
    assert int(cem.invalidity_margins_LR) == int(d['margins_LR'])
    assert int(cem.invalidity_margins_HR) == int(d['margins_HR'])
    m = cem.WrapArchitecture_PyTorch(torch.nn.Identity())
    np.testing.assert_array_equal(m.Conv_LR_with_Inv_hTh_OP.Filter_OP.weight.numpy(), d['w_inv'])
    np.testing.assert_array_equal(m.Upscale_OP.Filter_OP.weight.numpy(), d['w_up'])
    np.testing.assert_array_equal(m.DownscaleOP.Filter_OP.weight.numpy(), d['w_down'])
    assert cem.OP_names == ['Conv_LR_with_Inv_hTh_OP.Filter_OP', 'Upscale_OP.Filter_OP', 'DownscaleOP.Filter_OP']


def test_blurry_cubic_kernel_is_honoured():
    """The reference's sticky kernel cache ignores 'blurry_cubic_1' after a default init; here the
    kernel is an explicit argument, so it must change the design."""
    a = C.CEMnet(C.Get_CEM_Config(4))
    b = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel='blurry_cubic_1')
    assert b.ds_kernel.shape[0] > a.ds_kernel.shape[0]
    assert abs(b.ds_kernel.sum() - 1) < 1e-6


def _build(nb, latent, cem_mode, sf=4):
    net = esr_amd.RRDBNet(3, 3, 64, nb, upscale=sf, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    if cem_mode == 'none':
        return net
    return C.CEMnet(C.Get_CEM_Config(sf)).WrapArchitecture_PyTorch(net)


@pytest.mark.parametrize('name', golden_names('rrdb_'))
def test_state_dict_layout_matches_reference(name):
    d = golden(name)
    if 'kernel' in d:
        pytest.skip('layout identical to the bicubic case; filter sizes covered by the design test')
    ref = json.loads(str(d['keys']))
    m = _build(int(d['nb']), bool(int(d['latent'])), str(d['cem_mode']), fixture_upscale(d))
    ours = [(k, list(v.shape)) for k, v in m.state_dict().items()]
    assert ours == [(k, list(s)) for k, s in ref]


def test_rrdbnet_x3_raises_like_the_reference():
    """architecture.py:132-144: the reference's ×3 upsampler is an nn.Sequential concatenated to a list (TypeError);
    there is no ×3 model to match."""
    with pytest.raises(NotImplementedError):
        esr_amd.RRDBNet(3, 3, 64, 1, upscale=3, num_latent_channels=0)


def test_define_G_from_shipped_config():
    opt = {'gpu_ids': None, 'is_train': False, 'scale': 4,
           'network_G': {'which_model_G': 'RRDB_net', 'CEM_arch': 1, 'latent_input': 'all_layers',
                         'latent_input_domain': 'HR_downscaled', 'latent_channels': 3, 'norm_type': None,
                         'mode': 'CNA', 'nf': 64, 'nb': 23, 'in_nc': 3, 'out_nc': 3, 'gc': 32, 'group': 1},
           'datasets': {'train': {'patch_size': 256}}}
    cem = C.CEMnet(C.Get_CEM_Config(4))
    g = esr_amd.define_G(opt, CEM=cem, num_latent_channels=3)
    assert isinstance(g, C.CEM_PyTorch)
    assert sum(p.numel() for p in g.parameters()) == 17064869  # = reference latent RRDB-23 + CEM (fixture keys)
    g.eval()
    assert g.pre_pad
    g.train()
    assert not g.pre_pad


def test_pack_conv_weight_layout():
    torch.manual_seed(0)
    w = torch.randn(32, 67, 3, 3)
    cmap = [0, 1, 2] + [-1] * 5 + [3 + c for c in range(64)]
    pk = engine.pack_conv_weight(w, cmap, 32)
    assert pk.shape == (3, 9, 32, 32)
    for c in range(len(cmap)):
        j, cc = divmod(c, 32)
        for t in (0, 4, 8):
            if cmap[c] < 0:
                assert torch.all(pk[j, t, :, cc] == 0)
            else:
                assert torch.equal(pk[j, t, :, cc], w[:, cmap[c], t // 3, t % 3])
    assert torch.all(pk[2, :, :, 8:] == 0)  # channels >= 72 of the last chunk are padding


def test_upconv_polyphase_fold_equals_nearest_then_conv():
    """nearest-×2 then conv3×3 (block.py:294-301) == four 2×2 phase convs on the LR grid with folded taps."""
    torch.manual_seed(1)
    x = torch.randn(2, 5, 7, 6, dtype=torch.float64)
    w = torch.randn(4, 5, 3, 3, dtype=torch.float64)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode='nearest'), w, padding=1)
    out = torch.zeros_like(ref)
    xp = F.pad(x, (1, 1, 1, 1))
    for py in (0, 1):
        for px in (0, 1):
            wp = engine.fold_upconv_phase(w, py, px).to(torch.float64)
            # phase tap (a,b) reads LR offset (py+a-1, px+b-1): crop the padded input accordingly
            o = F.conv2d(xp[:, :, py:py + x.shape[2] + 1, px:px + x.shape[3] + 1], wp)
            out[:, :, py::2, px::2] = o
    assert torch.allclose(out, ref, atol=1e-12)


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(REPO, 'include', 'esr_amd.h')).read()
    declared = sorted(set(re.findall(r'^(?:int|int64_t|void|esr_timer_t)\s+(esr_\w+)\s*\(', hdr, flags=re.M)))
    assert declared and set(declared) == set(_lib.EXPORTED)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared:
        assert hasattr(lib, s), s
    assert _lib.load().esr_abi_version() == _lib.ABI_VERSION
    assert lib.esr_op_size() == ctypes.sizeof(_lib.EsrOp)  # op-list record layout matches the binding


def test_product_library_is_stateless():
    """The product library exports no kernel-selection setters (include/esr_amd.h: every entry point stateless); they
    exist only in the ablation library (csrc/esr_ablation.h), which also exports the whole product ABI."""
    syms = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True, text=True,
                          check=True).stdout
    exported = {line.split()[-1] for line in syms.splitlines() if line.split()[-1].startswith('esr_')}
    assert exported == set(_lib.EXPORTED), sorted(exported ^ set(_lib.EXPORTED))
    assert not any('_set_' in e for e in exported)
    if os.path.exists(_lib.ABLATION_PATH):
        abl = ctypes.CDLL(_lib.ABLATION_PATH)
        for name in _lib.EXPORTED + _lib.ABLATION_SETTERS:
            assert hasattr(abl, name), name
        hdr = open(os.path.join(REPO, 'explorable-super-resolution_old_amd', 'csrc', 'esr_ablation.h')).read()
        assert set(re.findall(r'^int\s+(esr_\w+)\s*\(', hdr, flags=re.M)) == set(_lib.ABLATION_SETTERS)


def test_product_path_refuses_cpu_tensors():
    net = _build(1, False, 'none')
    with torch.no_grad(), pytest.raises(RuntimeError, match='ROCm device'):
        net(torch.rand(1, 3, 8, 8))
    cem = _build(1, False, 'cem')
    with torch.no_grad(), pytest.raises(RuntimeError, match='ROCm device'):
        cem.DownscaleOP(torch.rand(1, 3, 8, 8))


def test_missing_library_fails_loudly(monkeypatch):
    monkeypatch.setattr(_lib, '_lib', None)
    monkeypatch.setattr(_lib, 'LIB_PATH', '/nonexistent/libesr_amd.so')
    with pytest.raises(_lib.ESRLibraryError):
        _lib.load()


def test_split_f16_roundtrip_and_x3_packing():
    torch.manual_seed(3)
    x = torch.randn(2, 3, 5, 24) * 10
    back = engine.from_split(engine.to_split(x))
    assert back.shape == x.shape
    # |v - hi - lo| <= 2^-22 |v|, or the f16 subnormal step (2^-24) once lo underflows
    assert bool(((back - x).abs() <= torch.maximum(2 ** -22 * x.abs(), torch.full_like(x, 2 ** -24))).all())
    w = torch.randn(32, 67, 3, 3) * 0.02
    pk = engine.pack_conv_weight(w, [0, 1, 2] + [-1] * 5 + [3 + c for c in range(64)], 32)
    px, scale = engine.pack_x3(pk)
    assert px.dtype == torch.float16 and px.shape == (6, 9, 32, 2, 2, 8)  # 16-channel K chunks
    assert math.log2(scale).is_integer() and 2 ** 14 <= float(pk.abs().max()) * scale < 2 ** 15
    rec16 = (px[..., 0, :].float() + px[..., 1, :].float()).reshape(6, 9, 32, 16) / scale
    rec = rec16.view(3, 2, 9, 32, 16).permute(0, 2, 3, 1, 4).reshape(pk.shape)
    assert float((rec - pk).abs().max()) <= 2 ** -22 * float(pk.abs().max())


@pytest.mark.parametrize('latent', [False, True])
def test_gather_plan_equals_direct_packing(latent):
    """The one-gather packing (GatherPlan) reproduces the per-conv packing for the forward weights, the rot180 /
    transposed / 0.2-scaled data-gradient weights, and maps the flat wgrad buffer back to reference-layout grads."""
    from esr_amd import train_engine as T
    torch.manual_seed(0)
    net = esr_amd.RRDBNet(3, 3, 64, 1, gc=32, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    for p in net.parameters():
        p.data.normal_()
    zc = 8 if latent else 0
    lr_map = (lambda n: list(range(n))) if not latent else (lambda n: [0, 1, 2] + [-1] * 5 + [3 + c for c in range(n)])
    pk = engine._packed(net, latent)
    conv = net.model[1].sub[0].RDB2.convs[3][0]
    assert torch.equal(pk.rdb[1][3].f32, engine.pack_conv_weight(conv.weight, lr_map(64 + 96), 32))
    assert torch.equal(pk.hr1.f32, engine.pack_conv_weight(net.model[6].weight, lr_map(64), 32))
    # refresh after an in-place update
    with torch.no_grad():
        conv.weight.mul_(3.0)
    pk = engine._packed(net, latent)
    assert torch.equal(pk.rdb[1][3].f32, engine.pack_conv_weight(conv.weight, lr_map(64 + 96), 32))
    # the upsampler phases: summed gathers, bitwise equal to folding then packing
    for row, (j, f) in zip(pk.up, engine.up_stages(net)):
        w = net.model[j][1].weight
        for cw, (py, px) in zip(row, [(a, b) for a in range(f) for b in range(f)]):
            assert torch.equal(cw.f32, engine.pack_conv_weight(engine.fold_upconv_phase(w, py, px, f),
                                                               list(range(64)), 64)), (j, py, px)
    bp = T._bwd_packed(net, latent)
    # fused RDB data-gradient weights: slice t's rows of rot180/transposed W_i, stacked over the convs i that read t
    rdb = net.model[1].sub[0].RDB3
    wfs = [rdb.convs[i][0].weight.detach().flip(2, 3).transpose(0, 1) for i in range(5)]
    for key, t0, nw, i_lo in (('x', zc, 64, 0), ('m3', zc + 128, 32, 3), ('m1', zc + 64, 32, 1)):
        blocks = []
        for i in range(i_lo, 5):
            cmap = lr_map(64 + 32 * i)
            blk = torch.zeros(nw, wfs[i].shape[1], 3, 3)
            for o in range(nw):
                if t0 + o < len(cmap) and cmap[t0 + o] >= 0:
                    blk[o] = wfs[i][cmap[t0 + o]]
            blocks.append(blk * 0.2 if i == 4 else blk)
        wt = torch.cat(blocks, 1)
        assert wt.shape[1] == 64 + 32 * (4 - i_lo)
        want = engine.pack_conv_weight(wt, list(range(wt.shape[1])), 32 if nw <= 32 else 64)
        assert torch.equal(bp.rdb_fused[2][key], want), key
    assert bp.rdb[2][4].slices == [] and ('z' in bp.rdb_fused[2]) == latent
    # wgrad buffer -> reference-layout gradient
    ref = {p: torch.randn_like(p) for p in net.parameters()}
    for b in [bp.first, bp.lr_conv, bp.hr0, bp.hr1] + bp.up + [c for r in bp.rdb for c in r]:
        g = ref[b.conv.weight]
        reg = torch.zeros(9, b.cin_pad, b.cout_pad)
        reg[:, b.ref_to_buf, :b.cout] = g.reshape(b.cout, -1, 9).permute(2, 1, 0)
        bp.dw[b.wg_off:b.wg_off + 9 * b.cin_pad * b.cout_pad] = reg.reshape(-1)
        bp.dw[b.wg_off + 9 * b.cin_pad * b.cout_pad:b.wg_off + 9 * b.cin_pad * b.cout_pad + b.cout] = ref[b.conv.bias]
    flat = bp.dw.index_select(0, bp.gidx)
    o = 0
    for p in bp.params:
        assert torch.equal(flat[o:o + p.numel()].view(p.shape), ref[p])
        o += p.numel()


@pytest.mark.parametrize('name', ['bicubic', 'learned13'])
def test_cem_batch_padding_and_kernels_match_reference(name):
    """Host parts of the CEM NumPy helpers: Pad_LR_Batch / Unpad_HR_Batch (data movement) and
    imresize(return_upscale_kernel=True), against the reference's outputs; the image resampling itself is a device
    path (tests/test_gpu_cem_np.py) and refuses to run without a GPU."""
    from esr_amd import imresize_CEM as I
    from oracle.recipe import synthetic_learned_kernel
    d = golden('cem_np_' + name)
    k = synthetic_learned_kernel() if name == 'learned13' else None
    cem = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=k)
    for key, v in (('pad1', cem.Pad_LR_Batch(d['lr_b'])), ('pad2', cem.Pad_LR_Batch(d['lr_b'], num_recursion=2)),
                   ('unpad1', cem.Unpad_HR_Batch(d['hr_b'])), ('unpad2', cem.Unpad_HR_Batch(d['hr_b'], 2)),
                   ('aa_up', I.imresize(None, [4], kernel=k, return_upscale_kernel=True)),
                   ('aa_down', I.imresize(None, [1 / 4], kernel=k, return_upscale_kernel=True))):
        assert v.shape == d[key].shape, key
        np.testing.assert_array_equal(v, d[key], err_msg=key)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match='no CPU path'):
            I.imresize(d['hr'], [1 / 4], kernel=k)
        with pytest.raises(RuntimeError, match='no CPU path'):
            cem.Project_2_kernel_subspace(d['hr'])


def test_cem_set_upscale_kernel_equals_fresh_design():
    from oracle.recipe import synthetic_learned_kernel
    k = synthetic_learned_kernel()
    a = C.CEMnet(C.Get_CEM_Config(4)).Set_Upscale_Kernel(k)
    b = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=k)
    for attr in ('ds_kernel', 'inv_hTh', 'invalidity_margins_LR', 'invalidity_margins_HR'):
        np.testing.assert_array_equal(getattr(a, attr), getattr(b, attr))
    net = esr_amd.RRDBNet(3, 3, 64, 1, num_latent_channels=0)
    cem = C.CEMnet(C.Get_CEM_Config(4))
    model = cem.WrapArchitecture_PyTorch(net, training_patch_size=384)
    cem.Set_Upscale_Kernel(k)
    model.Update_Filters(cem)
    fresh = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=k).WrapArchitecture_PyTorch(
        esr_amd.RRDBNet(3, 3, 64, 1, num_latent_channels=0), training_patch_size=384)
    sd, sf = model.state_dict(), fresh.state_dict()
    assert list(sd) == list(sf)
    for key in sd:
        if 'Filter' in key:
            np.testing.assert_array_equal(sd[key].numpy(), sf[key].numpy())
    assert (model.margins_LR, model.margins_HR) == (int(fresh.margins_LR), int(fresh.margins_HR)) != (10, 40)
    M = int(fresh.margins_HR)
    assert int(cem.loss_mask.sum()) == (384 - 2 * M) ** 2
    x = torch.arange(2 * 3 * 5 * 5, dtype=torch.float32).view(2, 3, 5, 5)
    assert torch.equal(model.LR_padder(x), fresh.LR_padder(x))


def test_lower_act_scale_counts_only_real_reductions():
    """at the floor A = 1 an overflow lowers nothing, so neither the counter nor a warning moves."""
    import warnings

    class Net:
        pass
    net = Net()
    net._esr_act_scale = 256.0
    r0 = engine.ACT_SCALE_REDUCTIONS
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        engine.lower_act_scale(net)
    assert net._esr_act_scale == 16.0 and engine.ACT_SCALE_REDUCTIONS == r0 + 1 and len(w) == 1
    net._esr_act_scale = 1.0
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        engine.lower_act_scale(net)
    assert net._esr_act_scale == 1.0 and engine.ACT_SCALE_REDUCTIONS == r0 + 1 and not w


def test_retired_switch_on_product_library_warns(monkeypatch):
    """an A/B environment switch of an earlier round does nothing on the product library; say so."""
    import warnings
    monkeypatch.setenv('ESR_DCONV_HALO', '0')
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        _lib.bind(_lib.LIB_PATH)
    assert any('ESR_DCONV_HALO' in str(x.message) for x in w)


def test_union_of_launch_intervals():
    """bench.py's roofline divides a tag's FLOPs by the union of its launch intervals (two streams overlap)."""
    from esr_amd import engine
    assert engine.union_ms([]) == 0.0
    assert engine.union_ms([(0.0, 1.0), (2.0, 3.0)]) == 2.0
    assert engine.union_ms([(0.0, 2.0), (1.0, 3.0), (2.5, 2.7)]) == 3.0
    assert engine.union_ms([(1.0, 4.0), (0.0, 1.0), (5.0, 6.0), (3.0, 5.5)]) == 6.0
