"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE (read-only at /root/reference) in this
container.  Run once here; only the small .npz outputs are committed.  The reference never travels to the GPU box.

    python tests/golden/make_golden.py

The reference does not import cleanly on this image; these in-memory shims make it importable without
writing anything under /root/reference:
  1. `cv2` is absent.  Only `cv2.resize(delta, INTER_CUBIC)` is used on the hot path (imresize_CEM.py:88-94,
     Cubic_Kernel).  We restate OpenCV's published INTER_CUBIC (OpenCV 4.x imgproc/resize.cpp: A = -0.75, half-pixel
     source coordinate fx = (x+0.5)*in/out - 0.5, 4 taps, BORDER_REFLECT_101).  For a delta image at scale 4 every
     coefficient is a dyadic rational, so float32/float64 evaluation is exact.
  2. `scipy.signal.gaussian` moved to `scipy.signal.windows.gaussian` in SciPy 1.15.
  3. `torchvision` is absent; architecture.py only imports it at module top.
  4. `torch.cuda.FloatTensor` is used to cast CEM filters (CEMnet.py:74,134); mapped to the CPU type.
Bytecode: the reference directory carries __pycache__/*.pyc files; we never load them (pycache_prefix redirect) and
never write any (dont_write_bytecode).
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
sys.pycache_prefix = '/tmp/esr_golden_pycache'

import numpy as np
import scipy.signal
import scipy.signal.windows
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference/codes'
sys.path.insert(0, REPO)
from oracle.recipe import seeded_params, seeded_inputs, synthetic_learned_kernel  # noqa: E402


def _cv2_resize_cubic(img, dsize, interpolation=None):
    """OpenCV INTER_CUBIC restated (see module docstring). img: 2-D float array; dsize=(W, H)."""
    A = -0.75
    img = np.asarray(img, dtype=np.float64)

    def coeffs(t):
        w0 = ((A * (t + 1) - 5 * A) * (t + 1) + 8 * A) * (t + 1) - 4 * A
        w1 = ((A + 2) * t - (A + 3)) * t * t + 1
        w2 = ((A + 2) * (1 - t) - (A + 3)) * (1 - t) * (1 - t) + 1
        return np.array([w0, w1, w2, 1.0 - w0 - w1 - w2])

    def reflect101(i, n):
        if n == 1:
            return 0
        while i < 0 or i >= n:
            i = -i if i < 0 else 2 * n - 2 - i
        return i

    def resize_1d(src_len, dst_len):
        m = np.zeros((dst_len, src_len))
        scale = src_len / dst_len
        for x in range(dst_len):
            fx = (x + 0.5) * scale - 0.5
            sx = int(np.floor(fx))
            c = coeffs(fx - sx)
            for k in range(4):
                m[x, reflect101(sx - 1 + k, src_len)] += c[k]
        return m

    W, H = dsize
    my = resize_1d(img.shape[0], H)
    mx = resize_1d(img.shape[1], W)
    return my @ img @ mx.T


def install_shims():
    cv2 = types.ModuleType('cv2')
    cv2.INTER_CUBIC = 2
    cv2.resize = _cv2_resize_cubic
    sys.modules['cv2'] = cv2
    scipy.signal.gaussian = scipy.signal.windows.gaussian
    tv = types.ModuleType('torchvision')
    sys.modules['torchvision'] = tv
    torch.cuda.FloatTensor = torch.FloatTensor
    torch.cuda.DoubleTensor = torch.DoubleTensor
    sys.path.insert(0, REF)


class FixedGen(nn.Module):
    """Stand-in generator for CEM-only fixtures: returns a preset HR tensor (CEMnet.py:183 calls it once)."""

    def __init__(self, out):
        super().__init__()
        self.out = out
        self.num_latent_channels = 0
        self.upscale = 4

    def forward(self, x):
        return self.out


def cem_fixture(CEMnet, name, kernel):
    conf = CEMnet.Get_CEM_Config(4)
    cem = CEMnet.CEMnet(conf, upscale_kernel=kernel)
    d = dict(ds_kernel=np.asarray(cem.ds_kernel), inv_hTh=np.asarray(cem.inv_hTh),
             ds_half=np.int64(cem.ds_kernel_invalidity_half_size_LR), inv_half=np.int64(cem.inv_hTh_invalidity_half_size),
             margins_LR=np.int64(cem.invalidity_margins_LR), margins_HR=np.int64(cem.invalidity_margins_HR))
    if isinstance(kernel, np.ndarray):
        d['input_kernel'] = kernel
    mLR = int(cem.invalidity_margins_LR)
    # CEM forward on fixed (gen, LR) pairs, train mode (no pre-pad) and eval mode (pre-pad), non-square on purpose.
    B, h, w = 2, 20, 24
    lr, _ = seeded_inputs(100, (B, 3, h, w))
    rng = np.random.default_rng(101)
    gen_train = rng.random((B, 3, 4 * h, 4 * w)).astype(np.float32)
    gen_eval = rng.random((B, 3, 4 * (h + 2 * mLR), 4 * (w + 2 * mLR))).astype(np.float32)
    for mode, gen in (('train', gen_train), ('eval', gen_eval)):
        m = cem.WrapArchitecture_PyTorch(FixedGen(torch.from_numpy(gen)))
        m.train(mode == 'train')
        with torch.no_grad():
            out = m(torch.from_numpy(lr)).numpy()
        d['fwd_%s_lr' % mode] = lr
        d['fwd_%s_gen' % mode] = gen
        d['fwd_%s_out' % mode] = out
    m = cem.WrapArchitecture_PyTorch(FixedGen(None))
    d['w_inv'] = m.Conv_LR_with_Inv_hTh_OP.Filter_OP.weight.detach().numpy()
    d['w_up'] = m.Upscale_OP.Filter_OP.weight.detach().numpy()
    d['w_down'] = m.DownscaleOP.Filter_OP.weight.detach().numpy()
    # DownscaleOP alone on an HR image (GUI.py:1289,1900 call it directly)
    hr = rng.random((B, 3, 4 * h, 4 * w)).astype(np.float32)
    with torch.no_grad():
        d['down_hr'] = hr
        d['down_out'] = m.DownscaleOP(torch.from_numpy(hr)).numpy()
    np.savez_compressed(os.path.join(HERE, 'cem_%s.npz' % name), **d)
    print('cem_%s: ds %s inv %s margins %d/%d' % (name, d['ds_kernel'].shape, d['inv_hTh'].shape, mLR,
                                                  int(cem.invalidity_margins_HR)))
    return cem


def rrdb_fixture(arch, CEMnet, name, nb, latent, lr_shape, seed, w_scale, cem_mode=None, z_mode='pixel', kernel=None,
                 sf=4):
    nl = 3 if latent else 0
    net = arch.RRDBNet(in_nc=3, out_nc=3, nf=64, nb=nb, gc=32, upscale=sf, norm_type=None, act_type='leakyrelu',
                       mode='CNA', upsample_mode='upconv',
                       latent_input='all_layers_HR_downscaled' if latent else None, num_latent_channels=nl)
    model = net
    cem = None
    if cem_mode is not None:
        cem = CEMnet.CEMnet(CEMnet.Get_CEM_Config(sf), upscale_kernel=kernel)
        model = cem.WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    named_shapes = [(k, tuple(v.shape)) for k, v in sd.items()]
    params = seeded_params(named_shapes, seed, w_scale=w_scale)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    B, _, h, w = lr_shape
    lr, z = seeded_inputs(seed + 1, lr_shape, (B, 3, sf * h, sf * w) if latent else None, z_mode=z_mode)
    x = torch.from_numpy(lr)
    if latent:  # SRRaGANModel.ConcatLatent (SRRaGAN_model.py:249-255): raw view of HR Z into 3·sf² LR-sized channels
        zt = torch.from_numpy(z)
        x = torch.cat([zt.contiguous().view(B, 3 * sf * sf, h, w), x], 1)
    if cem is not None:
        model.train(cem_mode == 'train')
    else:
        model.eval()
    with torch.no_grad():
        out = model(x).numpy()
    d = dict(lr=lr, out=out, nb=np.int64(nb), latent=np.int64(latent), seed=np.int64(seed), w_scale=np.float64(w_scale),
             cem_mode=np.str_(cem_mode or 'none'), keys=np.str_(json.dumps(named_shapes)))
    if sf != 4:
        d['upscale'] = np.int64(sf)
    if z is not None:
        d['z'] = z
    if isinstance(kernel, np.ndarray):
        d['kernel'] = kernel
    np.savez_compressed(os.path.join(HERE, 'rrdb_%s.npz' % name), **d)
    print('rrdb_%s: in %s out %s |out| %.4f params %d' % (name, tuple(x.shape), out.shape, np.abs(out).mean(),
                                                          sum(int(np.prod(s)) for _, s in named_shapes)))


GRAD_KEYS = ('model.0.weight', 'model.0.bias', 'model.1.sub.0.RDB1.convs.0.0.weight', 'model.1.sub.0.RDB1.convs.4.0.weight',
             'model.1.sub.0.RDB3.convs.2.0.weight', 'model.1.sub.0.RDB3.convs.4.0.bias', 'model.1.sub.1.weight',
             'model.2.1.weight', 'model.3.1.bias', 'model.4.weight', 'model.6.weight', 'model.6.bias')

# ×2 (architecture.py:113-136): one upconv, so HR_conv0 / HR_conv1 are model.3 / model.5
GRAD_KEYS_X2 = GRAD_KEYS[:7] + ('model.2.1.weight', 'model.2.1.bias', 'model.3.weight', 'model.5.weight',
                                'model.5.bias')


def grad_fixture(arch, CEMnet, name, latent, lr_shape, seed, w_scale, sf=4):
    """Training-step gradients (SRRaGAN_model.py:347-348, 529): CEM-wrapped RRDBNet(nb=1) in train mode, loss =
    Σ out·R with a seeded R; dumps the gradients of GRAD_KEYS (prefixed 'generated_image_model.')."""
    nl = 3 if latent else 0
    net = arch.RRDBNet(in_nc=3, out_nc=3, nf=64, nb=1, gc=32, upscale=sf, norm_type=None, act_type='leakyrelu',
                       mode='CNA', upsample_mode='upconv',
                       latent_input='all_layers_HR_downscaled' if latent else None, num_latent_channels=nl)
    model = CEMnet.CEMnet(CEMnet.Get_CEM_Config(sf)).WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    named_shapes = [(k, tuple(v.shape)) for k, v in sd.items()]
    params = seeded_params(named_shapes, seed, w_scale=w_scale)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    model.train(True)
    B, _, h, w = lr_shape
    lr, z = seeded_inputs(seed + 1, lr_shape, (B, 3, sf * h, sf * w) if latent else None, z_mode='image')
    x = torch.from_numpy(lr)
    if latent:
        x = torch.cat([torch.from_numpy(z).contiguous().view(B, 3 * sf * sf, h, w), x], 1)
    out = model(x)
    R = torch.from_numpy(np.random.default_rng(seed + 2).standard_normal(tuple(out.shape)).astype(np.float32))
    (out * R).sum().backward()
    named = dict(model.named_parameters())
    d = dict(lr=lr, R=R.numpy(), out=out.detach().numpy(), latent=np.int64(latent), seed=np.int64(seed),
             w_scale=np.float64(w_scale), keys=np.str_(json.dumps(named_shapes)), nb=np.int64(1))
    if sf != 4:
        d['upscale'] = np.int64(sf)
    if z is not None:
        d['z'] = z
    for k in GRAD_KEYS if sf == 4 else GRAD_KEYS_X2:
        d['grad:' + k] = named['generated_image_model.' + k].grad.numpy()
    np.savez_compressed(os.path.join(HERE, 'grad_%s.npz' % name), **d)
    print('grad_%s: %d grads, |g conv_first| %.3e' % (name, len(GRAD_KEYS), np.abs(d['grad:model.0.weight']).mean()))


def zgrad_fixture(arch, CEMnet, name, cem_mode, lr_shape, seed, w_scale, kernel=None, sf=4):
    """Z-optimisation gradients (Z_optimization.py:545-553, 574-630): generator frozen (requires_grad False), latent
    RRDBNet(nb=1) CEM-wrapped in `cem_mode`, loss = Σ out·R; dumps dL/dZ (HR latent, [B,3,sf·h,sf·w]) and dL/dLR."""
    net = arch.RRDBNet(in_nc=3, out_nc=3, nf=64, nb=1, gc=32, upscale=sf, norm_type=None, act_type='leakyrelu',
                       mode='CNA', upsample_mode='upconv', latent_input='all_layers_HR_downscaled',
                       num_latent_channels=3)
    model = CEMnet.CEMnet(CEMnet.Get_CEM_Config(sf), upscale_kernel=kernel).WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    named_shapes = [(k, tuple(v.shape)) for k, v in sd.items()]
    params = seeded_params(named_shapes, seed, w_scale=w_scale)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    model.train(cem_mode == 'train')
    for q in model.parameters():
        q.requires_grad = False
    B, _, h, w = lr_shape
    lr, z = seeded_inputs(seed + 1, lr_shape, (B, 3, sf * h, sf * w), z_mode='pixel')
    zt = torch.from_numpy(z).requires_grad_(True)
    lt = torch.from_numpy(lr).requires_grad_(True)
    out = model(torch.cat([zt.view(B, 3 * sf * sf, h, w), lt], 1))
    R = torch.from_numpy(np.random.default_rng(seed + 2).standard_normal(tuple(out.shape)).astype(np.float32))
    (out * R).sum().backward()
    d = dict(lr=lr, z=z, R=R.numpy(), out=out.detach().numpy(), dz=zt.grad.numpy(), dlr=lt.grad.numpy(),
             seed=np.int64(seed), w_scale=np.float64(w_scale), cem_mode=np.str_(cem_mode),
             keys=np.str_(json.dumps(named_shapes)), nb=np.int64(1), latent=np.int64(1))
    if sf != 4:
        d['upscale'] = np.int64(sf)
    if isinstance(kernel, np.ndarray):
        d['kernel'] = kernel
    np.savez_compressed(os.path.join(HERE, 'zgrad_%s.npz' % name), **d)
    print('zgrad_%s: |dz| %.3e |dlr| %.3e' % (name, np.abs(d['dz']).mean(), np.abs(d['dlr']).mean()))


# config 5 at its production grid: the latent RRDB-23 + CEM (eval, pre-pad) with the learned
# 13×13 kernel, B=8 × 128² LR; the reference computes images 0 and 7 of the batch (eval mode: images independent).
Z_GRID = dict(B=8, h=128, nb=23, seed=820, w_scale=0.1, images=[0, 7], proj=16)


def _digest(v, seed, idx, k):
    g = np.asarray(v, dtype=np.float64).ravel()
    return np.random.default_rng([seed, idx]).standard_normal((k, g.size)) @ g


def kernelgan_x4_kernel():
    """A ×4 blur kernel made by the reference's own KernelGAN post-processing (KernelGAN/util.py:123-182, train.py:19-21
    with conf.X4): post_process_k (zeroize all but the n_filtering = 40 largest taps, re-centre with kernel_shift) of a
    13×13 ×2 estimate (G_kernel_size = 13, configs.py:25, 41), then analytic_kernel (×2 -> ×4, 37×37 cropped to 25×25).
    KernelGAN's own training cannot run here (CUDA-only, needs an image dataset): its ×2 estimate is synthetic, an
    anisotropic Gaussian on a small positive floor from a seeded NumPy stream.  Saved to kernelgan_x4.npz."""
    import importlib.util
    np.int = int  # shim: kernel_shift (util.py:204) uses the np.int alias NumPy 2 removed
    spec = importlib.util.spec_from_file_location('kgan_util', os.path.join(REF, 'KernelGAN', 'util.py'))
    util = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(util)
    rng = np.random.default_rng(1313)
    raw = synthetic_learned_kernel(size=13, sigma=(0.9, 1.5), theta_deg=-25.0, shift=(0.4, 0.1))
    raw = raw + 2e-3 * rng.random(raw.shape) * raw.max()
    raw = (raw / raw.sum()).astype(np.float32)
    k2 = util.post_process_k(torch.from_numpy(raw), n=40)
    k4 = util.analytic_kernel(k2)
    np.savez_compressed(os.path.join(HERE, 'kernelgan_x4.npz'), raw_x2=raw, post_x2=k2, kernel_x4=k4)
    return k4


def zgrid_fixture(arch, CEMnet, kernel=None, fname='grid_c5_zgrad.npz'):
    """Z-optimisation input gradients (Z_optimization.py:545-630, generator frozen, loss = Σ out·R) at config 5's grid,
    float64 and float32: K seeded random projections + norms of dL/dZ, dL/dLR and of the output per image (the full
    float64 gradients are 6 MB per image).  RRDB.forward (block.py:262-270) runs under torch.utils.checkpoint so that
    the float64 activations fit this container: the same ops on the same values, recomputed in the backward."""
    import torch.utils.checkpoint as ckpt
    import models.modules.block as blk
    fwd = blk.RRDB.forward
    blk.RRDB.forward = lambda self, x: ckpt.checkpoint(fwd, self, x, use_reentrant=False)
    cfg = dict(Z_GRID)
    k = synthetic_learned_kernel() if kernel is None else kernel
    B, h, idx = cfg['B'], cfg['h'], cfg['images']
    lr, z = seeded_inputs(cfg['seed'] + 1, (B, 3, h, h), (B, 3, 4 * h, 4 * h), z_mode='pixel')
    R = np.random.default_rng(cfg['seed'] + 2).standard_normal((B, 3, 4 * h, 4 * h)).astype(np.float32)
    d = {'cfg': np.str_(json.dumps(cfg)), 'kernel': k}
    for tag, dtype in (('f64', torch.float64), ('f32', torch.float32)):
        net = arch.RRDBNet(in_nc=3, out_nc=3, nf=64, nb=cfg['nb'], gc=32, upscale=4, norm_type=None,
                           act_type='leakyrelu', mode='CNA', upsample_mode='upconv',
                           latent_input='all_layers_HR_downscaled', num_latent_channels=3)
        model = CEMnet.CEMnet(CEMnet.Get_CEM_Config(4), upscale_kernel=k).WrapArchitecture_PyTorch(net)
        sd = model.state_dict()
        named_shapes = [(n, tuple(v.shape)) for n, v in sd.items()]
        params = seeded_params(named_shapes, cfg['seed'], w_scale=cfg['w_scale'])
        model.load_state_dict({n: torch.from_numpy(v) for n, v in params.items()}, strict=False)
        model = model.to(dtype)
        model.eval()  # (CEM_PyTorch.train returns None)
        for q in model.parameters():
            q.requires_grad = False
        zt = torch.from_numpy(z[idx]).to(dtype).requires_grad_(True)
        lt = torch.from_numpy(lr[idx]).to(dtype).requires_grad_(True)
        out = model(torch.cat([zt.view(len(idx), 48, h, h), lt], 1))
        (out * torch.from_numpy(R[idx]).to(dtype)).sum().backward()
        for j, i in enumerate(idx):
            for name, v in (('dz', zt.grad[j]), ('dlr', lt.grad[j]), ('out', out.detach()[j])):
                v = v.double().numpy()
                d['%s_%s_proj:%d' % (tag, name, i)] = _digest(v, cfg['seed'] + {'dz': 10, 'dlr': 11, 'out': 12}[name],
                                                              i, cfg['proj'])
                d['%s_%s_norm:%d' % (tag, name, i)] = np.float64(np.linalg.norm(v))
        print('zgrid [%s]: |dz| %s' % (tag, [float(zt.grad[j].norm()) for j in range(len(idx))]), flush=True)
        del model, out, zt, lt
    blk.RRDB.forward = fwd
    np.savez_compressed(os.path.join(HERE, fname), **d)


def disc_fixture(arch, loss_mod, name, seed):
    """Discriminator_VGG_128_ (architecture.py:222-284) with nb = n_layers = 6 as the shipped train config builds it
    once define_D's TypeError is resolved, plus one WGAN-GP discriminator loss + gradients exactly as
    optimize_parameters forms them (SRRaGAN_model.py:378-399, non-relativistic, loss.py:202-263)."""
    torch.manual_seed(seed)
    D = arch.Discriminator_VGG_128_(in_nc=3, base_nf=64, norm_type='batch', act_type='leakyrelu', mode='CNA',
                                    input_patch_size=80, nb=6)
    sd = D.state_dict()
    named_shapes = [(k, tuple(v.shape)) for k, v in sd.items()]
    params = seeded_params([(k, s) for k, s in named_shapes if 'running' not in k and 'num_batches' not in k],
                           seed, w_scale=1.0)
    D.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    D.train()
    rng = np.random.default_rng(seed + 1)
    real = torch.from_numpy(rng.random((3, 3, 80, 72)).astype(np.float32))
    fake = torch.from_numpy(rng.random((3, 3, 80, 72)).astype(np.float32))
    rp = torch.from_numpy(rng.random((3, 1, 1, 1)).astype(np.float32))
    cri_gan = loss_mod.GANLoss('wgan-gp', 1.0, 0.0)
    cri_gp = loss_mod.GradientPenaltyLoss()
    pred_real = D(real)
    pred_fake = D(fake)
    l_d_real = 2 * cri_gan(pred_real, True)
    l_d_fake = 2 * cri_gan(pred_fake, False)
    interp = rp * fake + (1 - rp) * real
    interp.requires_grad = True
    l_d_gp = 10 * cri_gp(interp, D(interp))
    l_d_total = (l_d_real + l_d_fake) / 2 + l_d_gp
    l_d_total.backward()
    range_loss = loss_mod.CreateRangeLoss([0, 1])(torch.from_numpy((rng.random((2, 3, 8, 8)) * 1.6 - 0.3)
                                                                   .astype(np.float32)))
    d = dict(real=real.numpy(), fake=fake.numpy(), rp=rp.numpy(), pred_real=pred_real.detach().numpy(),
             pred_fake=pred_fake.detach().numpy(), l_d_real=l_d_real.item(), l_d_fake=l_d_fake.item(),
             l_d_gp=l_d_gp.item(), l_d_total=l_d_total.item(), range_loss=range_loss.item(), seed=np.int64(seed),
             keys=np.str_(json.dumps(named_shapes)), range_seed=np.int64(seed + 1))
    for k, p in D.named_parameters():
        d['grad:' + k] = p.grad.numpy()
    for k, v in D.state_dict().items():
        if 'running' in k:
            d['buf:' + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, 'disc_%s.npz' % name), **d)
    print('disc_%s: out %s, l_d_total %.5f (gp %.5f), %d params' % (name, pred_real.shape, l_d_total.item(),
                                                                   l_d_gp.item(), len(named_shapes)))


def cem_np_fixture(CEMnet, name, kernel):
    """The reference's NumPy image helpers (CEMnet.py:44-57,88-100; imresize_CEM.py:7-71) on HWC float64 images.
    Must run while imresize.kernels holds this CEMnet's kernel (the CEMnet constructor puts it there)."""
    from CEM.imresize_CEM import imresize
    cem = CEMnet.CEMnet(CEMnet.Get_CEM_Config(4), upscale_kernel=kernel)
    rng = np.random.default_rng(300 if kernel is None else 301)
    f32 = lambda *s: rng.random(s).astype(np.float32).astype(np.float64)  # noqa: E731 (exact in fp32)
    h, w = 20, 24
    lr, hr, hr2, gray = f32(h, w, 3), f32(4 * h, 4 * w, 3), f32(4 * h, 4 * w, 3), f32(4 * h, 4 * w)
    m = int(cem.invalidity_margins_LR)
    lr_b, hr_b = f32(2, h, w, 3), f32(2, 4 * (h + 4 * m), 4 * (w + 4 * m), 3)
    d = dict(lr=lr, hr=hr, hr2=hr2, gray=gray, lr_b=lr_b, hr_b=hr_b)
    d['down'] = imresize(hr, [1 / 4])
    d['down_zp'] = imresize(hr, [1 / 4], use_zero_padding=True)
    d['down_gray'] = imresize(gray, [1 / 4])
    d['up'] = imresize(lr, [4])
    d['up_zp'] = imresize(lr, [4], use_zero_padding=True)
    d['up_shape'] = imresize(lr, output_shape=[4 * h, 4 * w])
    d['dt_up'] = cem.DT_Satisfying_Upscale(lr)
    d['project'] = cem.Project_2_kernel_subspace(hr)
    d['enforce'] = cem.Enforce_DT_on_Image_Pair(lr, hr)
    d['enforce_same'] = cem.Enforce_DT_on_Image_Pair(hr2, hr)
    d['pad1'] = cem.Pad_LR_Batch(lr_b)
    d['pad2'] = cem.Pad_LR_Batch(lr_b, num_recursion=2)
    d['unpad1'] = cem.Unpad_HR_Batch(hr_b)
    d['unpad2'] = cem.Unpad_HR_Batch(hr_b, num_recursion=2)
    d['aa_up'] = imresize(None, [4], return_upscale_kernel=True)
    d['aa_down'] = imresize(None, [1 / 4], return_upscale_kernel=True)
    np.savez_compressed(os.path.join(HERE, 'cem_np_%s.npz' % name), **d)
    print('cem_np_%s: %s' % (name, {k: v.shape for k, v in d.items()}))


def main():
    install_shims()
    import CEM.CEMnet as CEMnet
    if sys.argv[1:] == ['cem_np']:  # only the NumPy-helper fixtures (bicubic first: imresize.kernels is sticky)
        cem_np_fixture(CEMnet, 'bicubic', None)
        cem_np_fixture(CEMnet, 'learned13', synthetic_learned_kernel())
        return
    import models.modules.architecture as arch
    torch.set_num_threads(8)
    if sys.argv[1:] == ['c5grid']:  # config 5's grid, learned kernel: its own process (imresize's sticky kernel)
        zgrid_fixture(arch, CEMnet)
        return
    if sys.argv[1:] == ['c5grid_kgan']:  # config 5's grid with the KernelGAN-recipe ×4 kernel (margins 22/88)
        zgrid_fixture(arch, CEMnet, kernelgan_x4_kernel(), 'grid_c5_zgrad_kgan.npz')
        return
    if sys.argv[1:] == ['scale2grad']:  # ×2 training and Z-optimisation gradients (own process: sticky bicubic)
        grad_fixture(arch, CEMnet, 'x2_plain_nb1', False, (2, 3, 12, 16), 70, 0.5, sf=2)
        grad_fixture(arch, CEMnet, 'x2_latent_nb1', True, (2, 3, 12, 12), 71, 0.5, sf=2)
        zgrad_fixture(arch, CEMnet, 'x2_eval', 'eval', (2, 3, 12, 12), 72, 0.5, sf=2)
        zgrad_fixture(arch, CEMnet, 'x2_train', 'train', (2, 3, 12, 16), 73, 0.5, sf=2)
        return
    if sys.argv[1:] == ['scale2']:  # ×2 generators (architecture.py:113-136) in their own process: imresize's bicubic
        sf = 2                     # kernel is process-global and sticky.  (×3 cannot be built by the reference:
        #                            architecture.py:144 concatenates a list and the ×3 nn.Sequential -> TypeError)
        rrdb_fixture(arch, CEMnet, 'x%d_plain_nb1' % sf, 1, False, (2, 3, 12, 16), 40 + sf, 0.5, sf=sf)
        rrdb_fixture(arch, CEMnet, 'x%d_plain_nb2_cem_eval' % sf, 2, False, (1, 3, 12, 14), 50 + sf, 0.5,
                     cem_mode='eval', sf=sf)
        rrdb_fixture(arch, CEMnet, 'x%d_latent_nb1_cem_eval' % sf, 1, True, (1, 3, 12, 12), 60 + sf, 0.5,
                     cem_mode='eval', sf=sf)
        return
    # --- CEM filter design + CEM forward, bicubic default then a learned (non-bicubic) kernel ---
    cem_fixture(CEMnet, 'bicubic', None)
    # --- RRDBNet plain / latent, bare and CEM-wrapped (bicubic kernel) ---
    rrdb_fixture(arch, CEMnet, 'plain_nb2', 2, False, (2, 3, 12, 16), 1, 0.1)
    rrdb_fixture(arch, CEMnet, 'plain_nb2_s1', 2, False, (2, 3, 12, 16), 2, 1.0)
    rrdb_fixture(arch, CEMnet, 'latent_nb2', 2, True, (2, 3, 12, 16), 3, 0.1)
    rrdb_fixture(arch, CEMnet, 'latent_nb2_s1', 2, True, (2, 3, 10, 14), 4, 1.0, z_mode='image')
    rrdb_fixture(arch, CEMnet, 'plain_nb1_cem_eval', 1, False, (1, 3, 12, 12), 5, 0.5, cem_mode='eval')
    rrdb_fixture(arch, CEMnet, 'plain_nb1_cem_train', 1, False, (2, 3, 12, 12), 6, 0.5, cem_mode='train')
    rrdb_fixture(arch, CEMnet, 'latent_nb1_cem_eval', 1, True, (1, 3, 12, 12), 7, 0.5, cem_mode='eval')
    rrdb_fixture(arch, CEMnet, 'latent_nb1_cem_train', 1, True, (2, 3, 12, 16), 8, 0.5, cem_mode='train')
    rrdb_fixture(arch, CEMnet, 'plain_nb23', 23, False, (1, 3, 16, 16), 9, 0.1)
    rrdb_fixture(arch, CEMnet, 'latent_nb23_cem_eval', 23, True, (1, 3, 16, 16), 10, 0.1, cem_mode='eval')
    rrdb_fixture(arch, CEMnet, 'plain_nb23_s1_cem_eval', 23, False, (1, 3, 16, 16), 11, 1.0, cem_mode='eval')
    # --- discriminator + WGAN-GP / range losses ---
    import models.modules.loss as loss_mod
    disc_fixture(arch, loss_mod, 'vgg128_nb6', 15)
    # --- training-step gradients (bicubic CEM, train mode) ---
    grad_fixture(arch, CEMnet, 'plain_nb1', False, (2, 3, 12, 16), 13, 0.5)
    grad_fixture(arch, CEMnet, 'latent_nb1', True, (2, 3, 12, 12), 14, 0.5)
    # --- Z-optimisation input gradients (frozen G) ---
    zgrad_fixture(arch, CEMnet, 'eval', 'eval', (2, 3, 12, 12), 16, 0.5)
    zgrad_fixture(arch, CEMnet, 'train', 'train', (2, 3, 12, 16), 17, 0.5)
    # --- learned kernel last: imresize.kernels is process-global and sticky (imresize_CEM.py:9,23-42) ---
    k = synthetic_learned_kernel()
    cem_fixture(CEMnet, 'learned13', k)
    rrdb_fixture(arch, CEMnet, 'latent_nb1_cem_eval_learned', 1, True, (1, 3, 12, 12), 12, 0.5, cem_mode='eval', kernel=k)
    zgrad_fixture(arch, CEMnet, 'eval_learned', 'eval', (1, 3, 12, 12), 18, 0.5, kernel=k)


if __name__ == '__main__':
    main()
