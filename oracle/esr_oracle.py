"""CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Functions cite the reference (paths relative to /root/reference/codes) they restate.  Convolutions use
torch.nn.functional.conv2d on CPU (the reference's own op, fp32); the CEM filter design uses NumPy float64 and
scipy.signal.convolve2d exactly like the reference.
"""
import numpy as np
import torch
import torch.nn.functional as F
from scipy.signal import convolve2d

LRELU = 0.2      # block.py:10 (act(neg_slope=0.2))
RES_SCALE = 0.2  # block.py:235 (RDB) and block.py:270 (RRDB)


# ----------------------------------------------------------------------------------------------------------------------
# CEM filter design (init-time, NumPy float64)
# ----------------------------------------------------------------------------------------------------------------------
def cubic_upscale_kernel(sf):
    """imresize_CEM.py:88-94 Cubic_Kernel: cv2 INTER_CUBIC image of a delta, cropped to its support.

    For an integer scale the 2-D kernel is the outer product of the 1-D OpenCV cubic weights (A=-0.75, half-pixel
    source coordinate).  The response at output x to a unit delta at input c is the cubic weight of tap (c - sx + 1)
    where fx = (x+0.5)/sf - 0.5, sx = floor(fx).
    """
    A = -0.75

    def w(t):  # cubic convolution kernel of distance t
        t = abs(t)
        if t <= 1:
            return ((A + 2) * t - (A + 3)) * t * t + 1
        if t < 2:
            return ((A * t - 5 * A) * t + 8 * A) * t - 4 * A
        return 0.0

    c = 5  # Delta_Im(11): delta at ceil(11/2)-1
    taps = []
    for x in range(sf * 11):
        fx = (x + 0.5) / sf - 0.5
        taps.append(w(fx - c))
    taps = np.array(taps)
    nz = np.nonzero(taps)[0]
    k1 = taps[nz[0]:nz[-1] + 1]
    return np.outer(k1, k1)


def _energy_distribution(k):
    """imresize_CEM.py:161-163."""
    e = [np.sqrt(np.sum(k ** 2))] + [np.sqrt(np.sum(k[f:-f, f:-f] ** 2)) for f in range(1, int(np.ceil(k.shape[0] / 2)))]
    return np.array(e) / e[0]


def center_mass(kernel, sf):
    """imresize_CEM.py:113-159: pad a custom kernel so its centroid sits in the middle, then trim to 99 % energy."""
    n = kernel.shape[0]
    xg, yg = np.meshgrid(np.arange(n), np.arange(n))
    xc = convolve2d(xg, kernel, mode='valid') + 1
    yc = convolve2d(yg, kernel, mode='valid') + 1
    x_pad, y_pad = 2 * (n / 2 - xc), 2 * (n / 2 - yc)
    diff = np.round(np.abs(y_pad)) - np.round(np.abs(x_pad))
    pre_x, post_x = np.maximum(0, -x_pad), np.maximum(0, x_pad)
    pre_y, post_y = np.maximum(0, -y_pad), np.maximum(0, y_pad)
    r = lambda v: int(np.round(v))  # noqa: E731

    def split(pre, post, d):
        off = np.round(post) - post - (np.round(pre) - pre)
        pre, post = r(pre), r(post)
        if off > 0:
            return pre + int(np.floor(d / 2)), post + int(np.ceil(d / 2))
        return pre + int(np.ceil(d / 2)), post + int(np.floor(d / 2))

    if diff > 0:
        pre_y, post_y = r(pre_y), r(post_y)
        pre_x, post_x = split(pre_x, post_x, diff)
    elif diff < 0:
        pre_x, post_x = r(pre_x), r(post_x)
        pre_y, post_y = split(pre_y, post_y, -diff)
    k = np.pad(kernel, ((r(pre_y), r(post_y)), (r(pre_x), r(post_x))))
    assert k.shape[0] == k.shape[1]
    m = np.argwhere(_energy_distribution(k) < 0.99)[0][0] * np.ones(2, dtype=np.int64)
    i = 0
    while np.mod(k.shape[0] - np.sum(m) - 1 + np.mod(sf + 1, 2), sf) != 0:
        m[i] -= 1
        i = (i + 1) % 2
    k = k[m[0]:-m[1], m[0]:-m[1]]
    return k / np.sum(k)


def upscale_kernel(sf, kernel=None):
    """imresize_CEM.py:18-47 with return_upscale_kernel=True: the (possibly custom) upscale kernel, zero-padded by the
    even-factor stride imbalance (calc_strides(None, sf): pre = sf-floor(sf/2)-1, post = floor(sf/2))."""
    post = sf // 2
    pre = sf - post - 1
    kpre, kpost = max(0, post - pre), max(0, pre - post)
    if kernel is None:
        k = cubic_upscale_kernel(sf)
    else:
        assert abs(1 - np.sum(kernel)) < np.finfo(np.float32).eps
        k = center_mass(np.rot90(kernel, 2), sf) * sf ** 2
    return np.pad(k, ((kpre, kpost), (kpre, kpost)))


def _margin(response, limit):
    """CEMnet.py:35-42: index past the deepest pixel whose normalised response deviates beyond `limit`."""
    n = response.shape[0]
    r = response / response[n // 2, n // 2]
    r[r <= 0] = limit / 2
    bad = np.exp(-np.abs(np.log(r))) < limit
    m = [np.argwhere(bad[:n // 2, n // 2])[-1][0] + 1, np.argwhere(bad[n // 2, :n // 2])[-1][0] + 1]
    return int(max(m))


def cem_design(sf=4, kernel=None, lower_magnitude_bound=0.01, perturbation_limit=0.999, energy=1 - 1e-6):
    """CEMnet.__init__ (CEMnet.py:17-26), Return_kernel (:218-219), compute_inv_hTh (:105-126)."""
    k_up = upscale_kernel(sf, kernel)
    ds = np.rot90(k_up, 2).astype(np.float32) / np.int32(sf ** 2)
    # ds_kernel margin: zero-padded imresize(ones, 1/sf) (imresize_CEM.py:44-45, 65-66, 70)
    aa = np.rot90(k_up * (1.0 / sf) ** 2, 2)
    pre = sf - sf // 2 - 1
    ones = convolve2d(np.ones((sf * 100, sf * 100)), aa, mode='same')[pre::sf, pre::sf]
    ds_half = _margin(ones, perturbation_limit)
    # hTh and its regularised inverse
    hTh = convolve2d(ds, np.rot90(ds, 2)) * sf ** 2
    half = np.ceil(np.array(hTh.shape) / 2)
    p0 = np.mod(half, sf)
    p0[p0 == 0] = sf
    p0 = (p0 - 1).astype(np.int64)
    hTh = hTh[p0[0]::sf, p0[1]::sf]
    H = np.fft.fft2(np.pad(hTh, 18))
    H = H * np.maximum(1, lower_magnitude_bound / np.abs(H))
    inv = np.real(np.fft.ifft2(1 / H))
    mr, mc = np.argmax(inv) // inv.shape[0], np.mod(np.argmax(inv), inv.shape[0])
    if not np.all(np.ceil(np.array(inv.shape) / 2) == np.array([mr, mc]) - 1):
        h = min(inv.shape[0] - mr - 1, inv.shape[0] - mc - 1, mr, mc)
        inv = inv[mr - h:mr + h + 1, mc - h:mc + h + 1]
    inv_half = _margin(convolve2d(np.ones((100, 100)), inv, mode='same'), perturbation_limit)
    drop = inv.shape[0] // 2 - _margin(convolve2d(np.ones((100, 100)), inv, mode='same'), energy)
    if drop > 0:
        inv = inv[drop:-drop, drop:-drop]
    m_lr = 2 * ds_half + inv_half
    return dict(ds_kernel=ds, inv_hTh=inv, ds_half=ds_half, inv_half=inv_half, margins_LR=m_lr, margins_HR=sf * m_lr,
                k_up=k_up, sf=sf)


# ----------------------------------------------------------------------------------------------------------------------
# CEM forward (CEM_PyTorch, CEMnet.py:142-194)
# ----------------------------------------------------------------------------------------------------------------------
def _dw(x, k, pad):
    """Depthwise (groups=3) cross-correlation with replicate padding (Filter_Layer, CEMnet.py:130-140)."""
    # the reference casts its filters to float32 (CEMnet.py:134); a float64 input (conditioning checks) keeps those values
    w = torch.as_tensor(np.ascontiguousarray(k), dtype=torch.float32).to(x.dtype)[None, None].repeat(x.shape[1], 1, 1, 1)
    return F.conv2d(F.pad(x, (pad, pad, pad, pad), mode='replicate'), w, groups=x.shape[1])


def cem_downscale(y, ds_kernel, sf=4):
    """DownscaleOP (CEMnet.py:152,157-162): replicate pad, xcorr with rot180(ds_kernel), keep phase pre_stride."""
    pre = sf - sf // 2 - 1
    return _dw(y, np.rot90(ds_kernel, 2), ds_kernel.shape[0] // 2)[:, :, pre::sf, pre::sf]


def cem_upscale(v, ds_kernel, sf=4):
    """Upscale_OP (CEMnet.py:153-159): zero-stuff at phase pre_stride, replicate pad, xcorr with sf²·ds_kernel."""
    pre = sf - sf // 2 - 1
    B, C, h, w = v.shape
    s = torch.zeros(B, C, sf * h, sf * w, dtype=v.dtype)
    s[:, :, pre::sf, pre::sf] = v
    return _dw(s, ds_kernel * sf ** 2, ds_kernel.shape[0] // 2)


def cem_inv(v, inv_hTh):
    """Conv_LR_with_Inv_hTh_OP (CEMnet.py:149-151)."""
    return _dw(v, inv_hTh, inv_hTh.shape[0] // 2)


def cem_forward(gen, lr, design, pre_pad, sf=4):
    """CEMnet.py:184-190 given the generator output `gen` (already computed on the padded input when pre_pad)."""
    ds, inv = design['ds_kernel'], design['inv_hTh']
    if pre_pad:
        m = design['margins_LR']
        lr = F.pad(lr, (m, m, m, m), mode='replicate')
    a = cem_upscale(cem_inv(lr, inv), ds, sf)
    b = cem_upscale(cem_inv(cem_downscale(gen, ds, sf), inv), ds, sf)
    out = a + gen - b
    if pre_pad:
        M = design['margins_HR']
        out = out[:, :, M:-M, M:-M]
    return out


# ----------------------------------------------------------------------------------------------------------------------
# CEM NumPy image helpers (CEMnet.py:44-57, 88-100; imresize_CEM.py:7-71), HWC float64 like the reference
# ----------------------------------------------------------------------------------------------------------------------
def imresize_np(im, scale, k_up, use_zero_padding=False):
    """imresize_CEM.py:7-71 for an integer up (scale = sf) or down (scale = 1/sf) factor, align_center=False, with the
    padded upscale kernel k_up passed explicitly (the reference reads it from its process-global cache)."""
    sf = int(round(max(scale, 1 / scale)))
    post = sf // 2
    pre = sf - post - 1
    aa = k_up if scale > 1 else np.rot90(k_up * scale ** 2, 2)                        # :43-45
    pad = np.array(aa.shape) // 2                                                      # :49
    squeeze = im.ndim < 3
    im = im[:, :, None] if squeeze else im
    out = []
    for c in range(im.shape[2]):
        x = im[:, :, c]
        if scale > 1:                                                                  # :57-63 zero-stuff, filter
            s = np.zeros((sf * x.shape[0], sf * x.shape[1]))
            s[pre::sf, pre::sf] = x
            x = s
        if use_zero_padding:
            y = convolve2d(x, aa, mode='same')
        else:
            y = convolve2d(np.pad(x, ((pad[0], pad[0]), (pad[1], pad[1])), mode='edge'), aa, mode='valid')
        out.append(y if scale > 1 else y[pre::sf, pre::sf])                            # :70
    out = np.stack(out, -1)
    return out[:, :, 0] if squeeze else out


def dt_satisfying_upscale(lr, design):
    """CEMnet.DT_Satisfying_Upscale (CEMnet.py:53-57): edge-pad, zero-padded 'same' convolution with inv_hTh,
    imresize ×sf (edge padding), unpad."""
    sf = design['sf']
    m = 2 * design['inv_half'] + design['ds_half']
    x = np.pad(lr, ((m, m), (m, m), (0, 0)), mode='edge')                              # Pad_Image, :221-222
    x = np.stack([convolve2d(x[:, :, c], design['inv_hTh'], mode='same') for c in range(x.shape[-1])], -1)
    y = imresize_np(x, sf, design['k_up'])
    M = sf * m
    return y[M:-M, M:-M, :]                                                            # Unpad_Image, :224-225


def project_2_kernel_subspace(hr, design):
    """CEMnet.py:98-100."""
    return dt_satisfying_upscale(imresize_np(hr, 1 / design['sf'], design['k_up']), design)


def enforce_dt_on_image_pair(lr_source, hr_input, design):
    """CEMnet.py:88-96: the image closest to hr_input whose downscale is lr_source (LR or already HR-sized)."""
    sf = design['sf']
    same = [a == b for a, b in zip(lr_source.shape, hr_input.shape)]
    lrs = [sf * a == b for a, b in zip(lr_source.shape, hr_input.shape)]
    assert all(a or b for a, b in zip(same, lrs))
    src = dt_satisfying_upscale(lr_source, design) if any(lrs) else project_2_kernel_subspace(lr_source, design)
    return hr_input - project_2_kernel_subspace(hr_input, design) + src


def pad_lr_batch(batch, m, num_recursion=1):
    """CEMnet.py:44-47 (NHWC, edge padding by the LR invalidity margin, repeated)."""
    for _ in range(num_recursion):
        batch = 1.0 * np.pad(batch, ((0, 0), (m, m), (m, m), (0, 0)), mode='edge')
    return batch


def unpad_hr_batch(batch, m, sf, num_recursion=1):
    """CEMnet.py:49-51 (Python slice semantics: an over-large margin yields an empty batch)."""
    r = sf ** num_recursion * m * num_recursion
    return batch[:, r:-r, r:-r, :]


# ----------------------------------------------------------------------------------------------------------------------
# RRDBNet forward (architecture.py:151-175, block.py)
# ----------------------------------------------------------------------------------------------------------------------
def _conv(x, P, key, act):
    y = F.conv2d(x, P[key + '.weight'], P[key + '.bias'], padding=1)
    return F.leaky_relu(y, LRELU) if act else y


def _rdb(x, P, pfx):
    """ResidualDenseBlock_5C.forward, ModuleList mode (block.py:230-235)."""
    feats = [x]
    for i in range(5):
        feats.append(_conv(torch.cat(feats, 1), P, '%s.convs.%d.0' % (pfx, i), act=i < 4))
    return feats[-1] * RES_SCALE + x[:, -64:]


def _rrdb(x, P, pfx, z):
    """RRDB.forward (block.py:262-270)."""
    out = _rdb(x, P, pfx + '.RDB1')
    if z is not None:
        out = torch.cat([z, out], 1)
    out = _rdb(out, P, pfx + '.RDB2')
    if z is not None:
        out = torch.cat([z, out], 1)
    out = _rdb(out, P, pfx + '.RDB3')
    return out * RES_SCALE + x[:, -64:]


def bilinear_down4(z_hr):
    """F.interpolate(scale 1/4, bilinear, align_corners=False) (architecture.py:157): src = 4i+1.5, i.e. the mean of
    the 2×2 block z[4i+1:4i+3, 4j+1:4j+3]."""
    a = z_hr[:, :, 1::4, 1::4]
    b = z_hr[:, :, 1::4, 2::4]
    c = z_hr[:, :, 2::4, 1::4]
    d = z_hr[:, :, 2::4, 2::4]
    return ((a * 0.5 + b * 0.5) * 0.5) + ((c * 0.5 + d * 0.5) * 0.5)


def rrdbnet_forward(x, P, nb, latent, sf=4):
    """RRDBNet.forward.  x: [B, 3, h, w] (plain) or [B, 3·sf²+3, h, w] (latent, HR Z as a raw view,
    SRRaGAN_model.py:252).  P: dict of reference-named parameters without the 'generated_image_model.' prefix.
    sf 4: two nearest-×2 upconvs; 2 / 3: one nearest-×2 / ×3 upconv (architecture.py:113-136)."""
    z_lr = z_hr = None
    if latent:
        zr, x = x[:, :-3], x[:, -3:]
        B, _, h, w = x.shape
        z_hr = zr.reshape(B, -1, sf * h, sf * w)
        z_lr = bilinear_down4(z_hr) if sf == 4 else \
            F.interpolate(z_hr, scale_factor=1 / sf, mode='bilinear', align_corners=False)
        x = torch.cat([z_lr, x], 1)
    fea = _conv(x, P, 'model.0', act=False)
    out = torch.cat([z_lr, fea], 1) if latent else fea
    for k in range(nb):                      # ShortcutBlock (block.py:85-96)
        if k > 0 and latent:
            out = torch.cat([z_lr, out], 1)
        out = _rrdb(out, P, 'model.1.sub.%d' % k, z_lr)
    if latent:
        out = torch.cat([z_lr, out], 1)
    out = fea + _conv(out, P, 'model.1.sub.%d' % nb, act=False)
    ups = [2, 2] if sf == 4 else [sf]
    for i, f in enumerate(ups):  # upconv_blcok: nearest ×f, conv, LReLU (block.py:294-301)
        out = _conv(F.interpolate(out, scale_factor=f, mode='nearest'), P, 'model.%d.1' % (2 + i), act=True)
    if latent:
        out = torch.cat([z_hr, out], 1)
    out = _conv(out, P, 'model.%d' % (2 + len(ups)), act=True)
    if latent:
        out = torch.cat([z_hr, out], 1)
    return _conv(out, P, 'model.%d' % (4 + len(ups)), act=False)


def sr_forward(x, P, nb, latent, design=None, pre_pad=False, sf=4):
    """CEM_PyTorch.forward wrapping RRDBNet (CEMnet.py:169-190); design=None means a bare RRDBNet."""
    if design is None:
        return rrdbnet_forward(x, P, nb, latent, sf)
    if pre_pad:
        mL, mH = design['margins_LR'], design['margins_HR']
        if latent:
            zr, lr = x[:, :-3], x[:, -3:]
            B, _, h, w = lr.shape
            z = F.pad(zr.reshape(B, -1, sf * h, sf * w), (mH, mH, mH, mH), mode='replicate')
            lr = F.pad(lr, (mL, mL, mL, mL), mode='replicate')
            x = torch.cat([z.reshape(B, -1, h + 2 * mL, w + 2 * mL), lr], 1)
        else:
            x = F.pad(x, (mL, mL, mL, mL), mode='replicate')
    gen = rrdbnet_forward(x, P, nb, latent, sf)
    lr = x[:, -3:]
    ds, inv = design['ds_kernel'], design['inv_hTh']
    out = cem_upscale(cem_inv(lr, inv), ds, sf) + gen - cem_upscale(cem_inv(cem_downscale(gen, ds, sf), inv), ds, sf)
    if pre_pad:
        M = design['margins_HR']
        out = out[:, :, M:-M, M:-M]
    return out


def strip_prefix(params):
    return {k[len('generated_image_model.'):] if k.startswith('generated_image_model.') else k: torch.as_tensor(v)
            for k, v in params.items()}


# ----------------------------------------------------------------------------------------------------------------------
# Discriminator_VGG_128_ (architecture.py:222-284) — the patch D of the training step, on torch.nn CPU convolutions
# ----------------------------------------------------------------------------------------------------------------------
def reference_discriminator(in_nc=3, nf=64, nb=6, num_2_strides=5):
    """The module tree of Discriminator_VGG_128_(norm 'batch', act 'leakyrelu', mode 'CNA'): conv_block layers
    (block.py:129-156: Conv2d, BatchNorm2d except the first, LeakyReLU(0.2)) with the 3x3-s1 / 4x4-s2 plan
    (architecture.py:226-260), then the pseudo-FC head conv 8x8 valid + BN + LReLU, LReLU, conv 1x1 + BN + LReLU
    (architecture.py:262-276).  Same state_dict keys as the reference; plain nn.Conv2d (CPU/any device)."""
    import torch.nn as nn

    def block(ci, co, k, s, norm, pad):
        mods = [nn.Conv2d(ci, co, kernel_size=k, stride=s, padding=pad, bias=True)]
        if norm:
            mods.append(nn.BatchNorm2d(co, affine=True))
        mods.append(nn.LeakyReLU(LRELU, True))
        return mods

    plan = [(in_nc, nf, 3, 1, False), (nf, nf, 4, 2, True), (nf, 2 * nf, 3, 1, True), (2 * nf, 2 * nf, 4, 2, True),
            (2 * nf, 4 * nf, 3, 1, True), (4 * nf, 4 * nf, 4, 2, True), (4 * nf, 8 * nf, 3, 1, True),
            (8 * nf, 8 * nf, 4, 2, True), (8 * nf, 8 * nf, 3, 1, True), (8 * nf, 8 * nf, 4, 2, True)]
    left = num_2_strides
    mods = []
    for ci, co, k, s, norm in plan[:nb]:
        if s == 2:
            s = 2 if left > 0 else 1
            left -= 1
        mods += block(ci, co, k, s, norm, (k - 1) // 2)
    nfeat = [m for m in mods if isinstance(m, nn.BatchNorm2d)][-1].num_features

    class _D(nn.Module):
        def __init__(self):
            super().__init__()
            self.features = nn.Sequential(*mods)
            self.classifier = nn.Sequential(nn.Sequential(*block(nfeat, min(100, nfeat), 8, 1, True, 0)),
                                            nn.LeakyReLU(LRELU, False),
                                            nn.Sequential(*block(min(100, nfeat), 1, 1, 1, True, 0)))

        def forward(self, x):
            return self.classifier(self.features(x))
    return _D()
